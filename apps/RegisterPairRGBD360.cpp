// RegisterPairRGBD360 — the reference's Registration/RegisterPairRGBD360.cpp:60-101 over the MI355X
// library: load two Frame360 archives, undistort, build the sphere cloud and the PbMap, register the
// PbMaps (25 planes, PLANAR_3DoF) and print the matched planes and the pose.  The GICP refinement and
// the PCL viewers of the reference are outside the hot path and not reproduced.
//   usage: RegisterPairRGBD360 <frame1.bin> <frame2.bin> [calib_dir]
#include <rgbd360/rgbd360.h>

#include <cmath>
#include <cstdio>
#include <string>

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <frame1.bin> <frame2.bin> [calib_dir]\n", argv[0]);
        return 1;
    }
    const std::string calib_dir = argc > 3 ? argv[3] : std::string(RGBD360_DATA_DIR) + "/calib";
    try {
        r360::Context ctx(0);
        r360::Calib360 calib(ctx);                                   // QVGA sensors (Calib360.h:73-77)
        calib.loadExtrinsicCalibration(calib_dir + "/Extrinsics");
        calib.loadIntrinsicCalibration(calib_dir + "/Intrinsics");
        std::printf("Create sphere 1\n");
        r360::Frame360 frame360_1(&calib);
        frame360_1.loadFrame(argv[1]);
        frame360_1.undistort();
        frame360_1.buildSphereCloud();
        frame360_1.getPlanes();
        std::printf("Create sphere 2\n");
        r360::Frame360 frame360_2(&calib);
        frame360_2.loadFrame(argv[2]);
        frame360_2.undistort();
        frame360_2.buildSphereCloud();
        frame360_2.getPlanes();
        r360::RegisterRGBD360 registerer(ctx, std::string(RGBD360_DATA_DIR) + "/config_files/configLocaliser_sphericalOdometry.ini");
        const bool good = registerer.RegisterPbMap(&frame360_1, &frame360_2, 25, r360::RegisterRGBD360::PLANAR_3DoF);
        std::printf("planes %zu / %zu, registration %s\n", frame360_1.planes.size(), frame360_2.planes.size(),
                    good ? "good" : "insufficient");
        for (const auto& kv : registerer.getMatchedPlanes()) std::printf("%u %u\n", kv.first, kv.second);
        const r360::Matrix4f P = registerer.getPose();
        std::printf("Distance %g\nPose\n", std::sqrt(P(0, 3) * P(0, 3) + P(1, 3) * P(1, 3) + P(2, 3) * P(2, 3)));
        for (int r = 0; r < 4; ++r) std::printf("%10.6f %10.6f %10.6f %10.6f\n", P(r, 0), P(r, 1), P(r, 2), P(r, 3));
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 2;
    }
    return 0;
}
