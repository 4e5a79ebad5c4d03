// Drop-in check: the reference's SphereGraphSLAM tracking loop (SLAM/SphereGraphSLAM.cpp:78-231) and the
// LoopClosure360 loop thread's registration of keyframes the main thread built (include/LoopClosure360.h:83-126,
// 273-330), compiled against the façade through include/rgbd360/compat.h with the reference's constructors and
// call sites.  Left out: the Map360 viewer, the PCL filters, the topological partitioning's CMatrix bookkeeping and
// the graph optimizer (not on the north-star path); Map360 is reduced to the members these call sites touch.
//   main thread  frames: new Frame360(&calib), loadFrame, undistort, buildSphereCloud, getPlanes, id, node
//                (stitchSphericalImage stays commented out, as in the reference, :110, :158);
//                tracking: RegisterPbMap(Map.vpSpheres[*compareSphereId], frame360, MAX_MATCH_PLANES,
//                PLANAR_ODOMETRY_3DoF); currentPose * getPose(); getPose().block(0,3,3,1).norm();
//                mmConnectionKFs[..][..] = pair<Matrix4f, Matrix<float,6,6>>(getPose(), getInfoMat());
//                getAreaMatched() / areaSource (:175-231)
//   loop thread  the LoopClosure360 object (its RegisterRGBD360 member constructed on the main thread, :85) runs on a
//                std::thread: RegisterPbMap(Map.vpSpheres[compareLocalIdx], newKF, 25, PLANAR_3DoF), the
//                minMatchesThreshold / areaThreshold gate, then RegisterPhotoICP align360 (created on the loop
//                thread) with setSourceFrame(keyframe sphere) / setTargetFrame(new sphere), alignFrames360(rotOffset *
//                relativePose * rotOffset.inverse(), PHOTO_DEPTH), getOptimalPose, getHessian, SSO (:297-321).  The
//                refinement runs whatever the gate says (printed), so the cross-thread dense path is always exercised.
//                The loop thread also builds a frame on its own default context (a Calib360() of its own) and hands
//                it to the main thread, which registers it after the loop thread has exited.
//   same thread  the main thread repeats the loop thread's calls with objects of its own: tests/test_gpu_dropin.py
//                requires identical output.
//   usage: sphere_graph_dropin <dir with sphere_images_<n>.bin> <first frame> <selectSample>
#include <rgbd360/compat.h>

#include <cmath>
#include <cstdlib>
#include <iomanip>
#include <iostream>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#define MAX_MATCH_PLANES 25

using namespace std;

static void print_mat(const char* tag, const float* v, int n) {
    cout << tag << ':' << setprecision(9);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) cout << ' ' << v[c * n + r];
    cout << setprecision(6) << '\n';
}
static void print_pose(const char* tag, const Eigen::Matrix4f& T) { print_mat(tag, T.data(), 4); }
static void print_info(const char* tag, const Eigen::Matrix<float, 6, 6>& M) { print_mat(tag, M.data(), 6); }

// the members of Map360 (include/Map360.h) these call sites use
struct Map360 {
    std::vector<Frame360*> vpSpheres;
    std::vector<Eigen::Matrix4f> vTrajectoryPoses, vOptimizedPoses;
    std::vector<float> vTrajectoryIncrements;
    std::vector<unsigned> vSelectedKFs;
    std::vector<std::set<unsigned> > vsAreas, vsNeighborAreas;
    std::map<unsigned, std::map<unsigned, std::pair<Eigen::Matrix4f, Eigen::Matrix<float, 6, 6> > > > mmConnectionKFs;
    unsigned currentArea = 0;
    std::mutex mapMutex;
    void addKeyframe(Frame360* sphere, Eigen::Matrix4f& pose) {   // Map360.h:90-96
        sphere->pose = pose;
        vpSpheres.push_back(sphere);
        vTrajectoryPoses.push_back(pose);
    }
};

// The registration calls of LoopClosure360::run (LoopClosure360.h:108-330) on one keyframe pair, as a struct so
// the main thread can repeat them on its own objects.
struct LoopCheck {
    RegisterRGBD360& registerer;
    const char* tag;
    void operator()(Frame360* kf, Frame360* newKF) {
        int minMatchesThreshold = 5;    // :114-115
        float areaThreshold = 15.0;
        RegisterPhotoICP align360;      // :120-124
        align360.setNumPyr(5);
        align360.useSaliency(false);
        align360.setGrayVariance(3.f / 255);
        float angleOffset = 157.5;
        Eigen::Matrix4f rotOffset = Eigen::Matrix4f::Identity(); rotOffset(1,1) = rotOffset(2,2) = cos(angleOffset*PI/180); rotOffset(1,2) = sin(angleOffset*PI/180); rotOffset(2,1) = -rotOffset(1,2);

        bool bGoodRegistration = registerer.RegisterPbMap(kf, newKF, 25, RegisterRGBD360::RegisterRGBD360::RegisterRGBD360::PLANAR_3DoF);
        const bool gate = bGoodRegistration && registerer.getMatchedPlanes().size() > minMatchesThreshold && registerer.getAreaMatched() > areaThreshold;
        cout << tag << " pbmap good " << bGoodRegistration << " matches " << registerer.getMatchedPlanes().size()
             << " area " << setprecision(9) << registerer.getAreaMatched() << " areaSource " << registerer.areaSource
             << setprecision(6) << " gate " << gate << '\n';
        Eigen::Matrix4f relativePose = registerer.getPose();
        print_pose((string(tag) + " pbmap pose").c_str(), relativePose);
        print_info((string(tag) + " pbmap info").c_str(), registerer.getInfoMat());

        // Refine registration (:305-314)
        align360.setSourceFrame(kf->sphereRGB, kf->sphereDepth); // The reference keyframe
        align360.setTargetFrame(newKF->sphereRGB, newKF->sphereDepth);
        Eigen::Matrix4f initTransf_dense = rotOffset * relativePose * rotOffset.inverse();
        align360.alignFrames360(initTransf_dense, RegisterPhotoICP::PHOTO_DEPTH);
        relativePose = rotOffset.inverse() * align360.getOptimalPose() * rotOffset;
        Eigen::Matrix<float,6,6> informationMatrix = align360.getHessian();
        print_pose((string(tag) + " dense pose").c_str(), relativePose);
        print_info((string(tag) + " dense hessian").c_str(), informationMatrix);
        cout << tag << " dense SSO " << setprecision(9) << align360.SSO << setprecision(6) << '\n';
    }
};

class LoopClosure360 {
  public:
    Map360& Map;
    RegisterRGBD360 registerer;
    Frame360* built_here = nullptr;     // a frame built on the loop thread's own default context
    Calib360* calib_here = nullptr;
    std::string frame_file;

    LoopClosure360(Map360& map, const std::string& file)
        : Map(map), registerer(mrpt::format("%s/config_files/configLocaliser_sphericalOdometry.ini", PROJECT_SOURCE_PATH)),
          frame_file(file) {
        thread_hd_ = std::thread(&LoopClosure360::run, this);
    }
    void join() { if (thread_hd_.joinable()) thread_hd_.join(); }
    ~LoopClosure360() { join(); }

  private:
    std::thread thread_hd_;
    void run() {
        try {
            Frame360* kf;
            Frame360* newKF;
            {
                std::lock_guard<std::mutex> lk(Map.mapMutex);
                kf = Map.vpSpheres[0];
                newKF = Map.vpSpheres[1];
            }
            LoopCheck{registerer, "lc"}(kf, newKF);
            // a frame built here, on this thread's default context, outlives the thread
            calib_here = new Calib360();
            calib_here->loadExtrinsicCalibration();
            calib_here->loadIntrinsicCalibration();
            built_here = new Frame360(calib_here);
            built_here->loadFrame(frame_file);
            built_here->undistort();
            built_here->buildSphereCloud();
            built_here->getPlanes();
        } catch (const std::exception& e) {
            cout << "lc error: " << e.what() << '\n';
        }
    }
};

class SphereGraphSLAM {
  private:
    Map360 Map;

  public:
    ~SphereGraphSLAM() {
        for (unsigned i = 0; i < Map.vpSpheres.size(); i++) delete Map.vpSpheres[i];
    }

    int run(string path, int frame, const int& selectSample) {
        Map.currentArea = 0;
        Calib360 calib;
        calib.loadExtrinsicCalibration();
        calib.loadIntrinsicCalibration();
        RegisterRGBD360 registerer(mrpt::format("%s/config_files/configLocaliser_sphericalOdometry.ini", PROJECT_SOURCE_PATH));

        int frameOrder = 0;
        int numCheckRegistration = 5;
        unsigned noAssoc_threshold = 40;
        Eigen::Matrix4f currentPose = Eigen::Matrix4f::Identity();
        string fileName = path + mrpt::format("/sphere_images_%d.bin", frame);

        // Load first frame (:106-129)
        Frame360* frame360 = new Frame360(&calib);
        frame360->loadFrame(fileName);
        frame360->undistort();
//        frame360->stitchSphericalImage();
        frame360->buildSphereCloud();
        frame360->getPlanes();
        frame360->id = frameOrder;
        frame360->node = Map.currentArea;
        Map.addKeyframe(frame360, currentPose);
        Map.vOptimizedPoses.push_back(currentPose);
        Map.vSelectedKFs.push_back(0);
        Map.vTrajectoryIncrements.push_back(0);
        Map.vsAreas.push_back(std::set<unsigned>());
        Map.vsAreas[Map.currentArea].insert(frameOrder);
        Map.vsNeighborAreas.push_back(std::set<unsigned>());
        Map.vsNeighborAreas[Map.currentArea].insert(Map.currentArea);
        std::map<std::pair<int, int>, float> vSSO;
        cout << "planes " << frame360->planes.vPlanes.size() << '\n';

        frame += selectSample;
        fileName = path + mrpt::format("/sphere_images_%d.bin", frame);
        int tracked = 0;
        while (fexists(fileName.c_str())) {
            cout << "Frame " << fileName << endl;
            frame360 = new Frame360(&calib);
            frame360->loadFrame(fileName);
            frame360->undistort();
//        frame360->stitchSphericalImage();
            frame360->buildSphereCloud();
            frame360->getPlanes();
            frame360->id = ++frameOrder;
            frame360->node = Map.currentArea;
            int newLocalFrameID = Map.vsAreas[Map.currentArea].size();
            cout << "planes " << frame360->planes.vPlanes.size() << '\n';

            int compareLocalIdx = newLocalFrameID - 1;
            unsigned noAssoc = 0;
            bool frameRegistered = false;
            set<unsigned>::reverse_iterator compareSphereId = Map.vsAreas[Map.currentArea].rbegin();
            while (compareLocalIdx >= 0 && (compareLocalIdx >= newLocalFrameID - numCheckRegistration) && noAssoc < noAssoc_threshold) {
                std::cout << "Register  " << frame360->id << " with " << compareLocalIdx << std::endl;
                if (registerer.RegisterPbMap(Map.vpSpheres[*compareSphereId], frame360, MAX_MATCH_PLANES, RegisterRGBD360::PLANAR_ODOMETRY_3DoF)) {
                    cout << "Good TRACKING between " << frameOrder << " " << *compareSphereId << endl;
                    currentPose = currentPose * registerer.getPose();
                    Map.vTrajectoryIncrements.push_back(Map.vTrajectoryIncrements.back() + registerer.getPose().block(0,3,3,1).norm());
                    {std::lock_guard<std::mutex> updateLock(Map.mapMutex);
                        Map.addKeyframe(frame360, currentPose);
                        Map.vOptimizedPoses.push_back( Map.vOptimizedPoses.back() * registerer.getPose() );
                        Map.mmConnectionKFs[frameOrder] = std::map<unsigned, std::pair<Eigen::Matrix4f, Eigen::Matrix<float,6,6> > >();
                        Map.mmConnectionKFs[frameOrder][*compareSphereId] = std::pair<Eigen::Matrix4f, Eigen::Matrix<float,6,6> >(registerer.getPose(), registerer.getInfoMat());
                        Map.vsAreas[Map.currentArea].insert(frameOrder);
                    }
                    frameRegistered = true;
                    vSSO[std::make_pair(newLocalFrameID, compareLocalIdx)] = registerer.getAreaMatched() / registerer.areaSource;
                    // (what mmConnectionKFs received; *compareSphereId, a reverse iterator, names the new frame since
                    // the insert above)
                    print_pose("track pose", registerer.getPose());
                    print_info("track info", registerer.getInfoMat());
                    cout << "track SSO " << setprecision(9) << vSSO[std::make_pair(newLocalFrameID, compareLocalIdx)]
                         << " increment " << Map.vTrajectoryIncrements.back() << setprecision(6) << '\n';
                    print_pose("current", currentPose);
                    ++tracked;
                    break;
                }
                cout << "  Cannot associate to previous frame\n";
                ++noAssoc;
                --compareLocalIdx;
                ++compareSphereId;
            }
            if (!frameRegistered) {
                cout << "  No registration available for " << fileName << endl;
                delete frame360;
                --frameOrder;
            }
            frame += selectSample;
            fileName = path + mrpt::format("/sphere_images_%d.bin", frame);
        }
        cout << tracked << " tracked\n";
        if (Map.vpSpheres.size() < 2) return 4;

        // the loop thread registers the first two keyframes (built above, on this thread)
        LoopClosure360 loopCloser(Map, path + mrpt::format("/sphere_images_%d.bin", frame - selectSample));
        loopCloser.join();
        if (!loopCloser.built_here) return 5;

        // the same calls on this thread with its own objects
        RegisterRGBD360 registerer2(mrpt::format("%s/config_files/configLocaliser_sphericalOdometry.ini", PROJECT_SOURCE_PATH));
        LoopCheck{registerer2, "st"}(Map.vpSpheres[0], Map.vpSpheres[1]);

        // the frame the exited loop thread built (its context kept alive by the frame), registered here
        bool good = registerer.RegisterPbMap(Map.vpSpheres[0], loopCloser.built_here, MAX_MATCH_PLANES, RegisterRGBD360::PLANAR_ODOMETRY_3DoF);
        cout << "lt pbmap good " << good << " planes " << loopCloser.built_here->planes.vPlanes.size() << '\n';
        print_pose("lt pbmap pose", registerer.getPose());
        delete loopCloser.built_here;
        delete loopCloser.calib_here;
        return 0;
    }
};

int main(int argc, char** argv) {
    if (argc != 4) {
        cerr << "usage: " << argv[0] << " <pathToRawRGBDImagesDir> <firstFrame> <sampleStream>\n";
        return 1;
    }
    try {
        SphereGraphSLAM rgbd360_reg_seq;
        return rgbd360_reg_seq.run(argv[1], atoi(argv[2]), atoi(argv[3]));
    } catch (const std::exception& e) {
        cerr << "error: " << e.what() << '\n';
        return 2;
    }
}
