// Drop-in check: the reference's OdometryRGBD360 call sequence (Registration/OdometryRGBD360.cpp) compiled
// against the façade through include/rgbd360/compat.h, with the reference's own constructors and default
// arguments.  Only what the façade cannot provide is left out: the Map360 viewer, the PCL filters and the
// commented-out GICP (not on the north-star path).  The calls, in the reference's order:
//   construction  :60-73   RegisterRGBD360 registerer(ini); Calib360 calib; loadExtrinsicCalibration();
//                          loadIntrinsicCalibration()
//   first frame   :83-95   new Frame360(&calib), loadFrame, undistort, stitchSphericalImage, buildSphereCloud,
//                          getPlanes; RegisterPhotoICP align360; setNumPyr(5); useSaliency(false);
//                          setGrayVariance(3.f/255)
//   rotOffset     :138-139
//   per frame     :141-257 RegisterPbMap(frame360_1, frame360_2, MAX_MATCH_PLANES, PLANAR_3DoF); getPose();
//                          setTargetFrame / setSourceFrame(sphereRGB, sphereDepth); alignFrames360(rigidTransf_dense,
//                          PHOTO_DEPTH); rotOffset.inverse() * getOptimalPose() * rotOffset; the 0.4 m skip;
//                          currentPose = currentPose * rigidTransf
// Output (parsed by tests/test_gpu_dropin.py): per registered frame the PbMap verdict and pose, the dense pose
// (getOptimalPose) and the composed current pose.
//   usage: odometry_dropin <dir with sphere_images_<n>.bin> <first frame> <selectSample>
#include <rgbd360/compat.h>

#include <cmath>
#include <cstdlib>
#include <iomanip>
#include <iostream>
#include <string>

#define MAX_MATCH_PLANES 25

using namespace std;

static void print_pose(const char* tag, const Eigen::Matrix4f& T) {
    cout << tag << ':' << setprecision(9);
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) cout << ' ' << T(r, c);
    cout << setprecision(6) << '\n';
}

class Odometry360 {
  private:
    RegisterRGBD360 registerer;
    Calib360 calib;
    Frame360 *frame360_1 = nullptr, *frame360_2 = nullptr;

  public:
    Odometry360() : registerer(mrpt::format("%s/config_files/configLocaliser_sphericalOdometry.ini", PROJECT_SOURCE_PATH)) {
        calib.loadExtrinsicCalibration();
        calib.loadIntrinsicCalibration();
    }

    int run(const string& path_dataset, unsigned frame, int selectSample) {
        string fileName = path_dataset + mrpt::format("/sphere_images_%d.bin", frame);
        frame360_2 = new Frame360(&calib);
        frame360_2->loadFrame(fileName);
        frame360_2->undistort();
        frame360_2->stitchSphericalImage();
        frame360_2->buildSphereCloud();
        frame360_2->getPlanes();

        RegisterPhotoICP align360;
        align360.setNumPyr(5);
        align360.useSaliency(false);
        align360.setGrayVariance(3.f / 255);

        bool bGoodRegistration = true;
        Eigen::Matrix4f currentPose = Eigen::Matrix4f::Identity();
        frame += selectSample;
        fileName = mrpt::format("%s/sphere_images_%d.bin", path_dataset.c_str(), frame);
        Eigen::Matrix4f rigidTransf = Eigen::Matrix4f::Identity();
        Eigen::Matrix4f rigidTransf_pbmap = Eigen::Matrix4f::Identity();
        Eigen::Matrix4f rigidTransf_dense = Eigen::Matrix4f::Identity();
        float angleOffset = 157.5;
        Eigen::Matrix4f rotOffset = Eigen::Matrix4f::Identity();
        rotOffset(1, 1) = rotOffset(2, 2) = cos(angleOffset * PI / 180);
        rotOffset(1, 2) = sin(angleOffset * PI / 180);
        rotOffset(2, 1) = -rotOffset(1, 2);

        int registered = 0;
        while (fexists(fileName.c_str())) {
            cout << "Frame " << fileName << endl;
            if (bGoodRegistration) {
                if (frame360_1 != frame360_2) delete frame360_1;
                frame360_1 = frame360_2;
            } else if (frame360_2 != frame360_1) {
                delete frame360_2;   // the reference leaks the rejected frame here
            }
            frame360_2 = new Frame360(&calib);
            frame360_2->loadFrame(fileName);
            frame360_2->undistort();
            frame360_2->stitchSphericalImage();
            frame360_2->buildSphereCloud();
            frame360_2->getPlanes();

            bGoodRegistration = registerer.RegisterPbMap(frame360_1, frame360_2, MAX_MATCH_PLANES, RegisterRGBD360::PLANAR_3DoF);
            if (!bGoodRegistration)
                cout << "\tBad registration\n";
            else
                rigidTransf_pbmap = registerer.getPose();
            print_pose(bGoodRegistration ? "pbmap good" : "pbmap bad", registerer.getPose());

            align360.setTargetFrame(frame360_1->sphereRGB, frame360_1->sphereDepth);
            align360.setSourceFrame(frame360_2->sphereRGB, frame360_2->sphereDepth);
            align360.alignFrames360(rigidTransf_dense, RegisterPhotoICP::PHOTO_DEPTH);
            print_pose("dense optimal", align360.getOptimalPose());
            rigidTransf_dense = rotOffset.inverse() * align360.getOptimalPose() * rotOffset;
            rigidTransf = rigidTransf_dense;
            ++registered;

            float dist = rigidTransf.block(0, 3, 3, 1).norm();
            cout << "dist " << dist << endl;
            if (dist < 0.4) {
                bGoodRegistration = false;
                delete frame360_2;
                frame360_2 = frame360_1;
                frame += selectSample;
                fileName = path_dataset + mrpt::format("/sphere_images_%d.bin", frame);
                continue;
            }
            currentPose = currentPose * rigidTransf;
            print_pose("current", currentPose);
            rigidTransf_dense = Eigen::Matrix4f::Identity();
            frame += selectSample;
            fileName = path_dataset + mrpt::format("/sphere_images_%d.bin", frame);
        }
        if (frame360_1 != frame360_2) delete frame360_1;
        delete frame360_2;
        cout << registered << " registrations\n";
        return registered > 0 ? 0 : 4;
    }
};

int main(int argc, char** argv) {
    if (argc != 4) {
        cerr << "usage: " << argv[0] << " <pathToRawRGBDImagesDir> <firstFrame> <sampleStream>\n";
        return 1;
    }
    try {
        Odometry360 odometry360;
        return odometry360.run(argv[1], unsigned(atoi(argv[2])), atoi(argv[3]));
    } catch (const std::exception& e) {
        cerr << "error: " << e.what() << '\n';
        return 2;
    }
}
