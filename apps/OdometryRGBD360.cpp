// OdometryRGBD360 — the reference's Registration/OdometryRGBD360.cpp / OdometryKeyFrame360.cpp loop over
// the MI355X library: for each new Frame360, PbMap registration against the previous keyframe, dense
// RegisterPhotoICP refinement initialised with the rotOffset-conjugated PbMap pose (Register()), the
// |t| < 0.4 m frame skip (:230-238) and the trajectory prefix product currentPose *= rigidTransf (:257).
// As in the reference, the keyframe (frame360_1) advances only after a registration whose PbMap stage
// succeeded and whose dense translation reached 0.4 m (bGoodRegistration, :145-148, :189, :230-238).
//   usage: OdometryRGBD360 <dir with sphere_images_<n>.bin> [first] [step] [calib_dir]
//          OdometryRGBD360 --synthetic <n_frames> [skip]  (procedural room, 8 x 480x640, no I/O; skip = 1
//                                                          applies the |t| < 0.4 m frame skip, 0 registers
//                                                          every consecutive pair)
//          OdometryRGBD360 --throughput <n_frames> [repeats] [pipelines]
//                                                         (every consecutive pair of the synthetic sequence through
//                                                          the library's pipelined sequence runner, r360_sequence:
//                                                          the benchmark's configuration; prints pairs/s and the
//                                                          composed trajectory's end pose)
#include <rgbd360/rgbd360.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <memory>
#include <string>
#include <sys/stat.h>
#include <vector>

static bool fexists(const std::string& p) { struct stat st; return stat(p.c_str(), &st) == 0; }

// The benchmark's configuration from C++ (bench.py drives the same runner): frames rendered into page-locked host
// memory, uploaded per pair inside the timed region, `repeats` passes over all pairs after one warm-up pass.
static int throughput(int n_frames, int repeats, int pipelines) {
    r360_sequence_params sp;
    r360_sequence_default_params(&sp);
    if (pipelines > 0) sp.pipelines = pipelines;
    const int pairs = n_frames - 1;
    if (pairs < 1) { std::fprintf(stderr, "need at least 2 frames\n"); return 1; }
    sp.pipelines = std::min(sp.pipelines, std::max(1, pairs / 6));   // runs of >= 6 pairs (bench.py --min-run)
    const size_t nb = size_t(8) * sp.rows * sp.cols * 3, nd = size_t(8) * sp.rows * sp.cols;
    std::vector<uint8_t> bgr(nb * n_frames);
    std::vector<uint16_t> dep(nd * n_frames);
    const uint32_t seed = 360u << 16;
    std::vector<float> rt(128);
    for (int k = 0; k < 8; ++k) {                       // the shipped extrinsics, column-major
        const std::string p = std::string(RGBD360_DATA_DIR) + "/calib/Extrinsics/Rt_0" + std::to_string(k + 1) + ".txt";
        FILE* f = std::fopen(p.c_str(), "r");
        if (!f) { std::fprintf(stderr, "cannot read %s\n", p.c_str()); return 1; }
        float m[16];
        for (int i = 0; i < 16; ++i) if (std::fscanf(f, "%f", &m[i]) != 1) m[i] = 0;
        std::fclose(f);
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) rt[16 * k + c * 4 + r] = m[r * 4 + c];
    }
    for (int i = 0; i < n_frames; ++i) {
        float P[16];
        r360_synth_path_pose(seed, i, P);
        r360::check(r360_synth_frame_rt(sp.rows, sp.cols, rt.data(), seed, P, bgr.data() + nb * i, dep.data() + nd * i),
                    "synth_frame_rt");
    }
    r360::check(r360_host_register(bgr.data(), bgr.size()), "host_register");
    r360::check(r360_host_register(dep.data(), dep.size() * 2), "host_register");
    std::vector<const void*> pb(n_frames), pd(n_frames);
    for (int i = 0; i < n_frames; ++i) { pb[i] = bgr.data() + nb * i; pd[i] = dep.data() + nd * i; }
    r360_sequence* s = nullptr;
    r360::check(r360_sequence_create(0, &sp, nullptr, &s), "r360_sequence_create");
    std::vector<float> rec(size_t(std::max(repeats, 1)) * pairs * R360_SEQ_RECORD);
    r360::check(r360_sequence_run(s, 0, pairs, pb.data(), pd.data(), 0, 1, nullptr, 0, rec.data()), "warm-up");
    const auto t0 = std::chrono::steady_clock::now();
    r360::check(r360_sequence_run(s, 0, pairs, pb.data(), pd.data(), 0, repeats, nullptr, 0, rec.data()), "run");
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    r360_sequence_destroy(s);
    r360_host_unregister(bgr.data());
    r360_host_unregister(dep.data());
    r360::Matrix4f T;                                   // currentPose = currentPose * rigidTransf (:257)
    int failed = 0;
    for (int i = 0; i < pairs; ++i) {
        r360::Matrix4f M;
        std::memcpy(M.data(), &rec[size_t(i) * R360_SEQ_RECORD], sizeof(float) * 16);
        failed += rec[size_t(i) * R360_SEQ_RECORD + 52] != 0.f;
        T = T * M;
    }
    std::printf("%d pairs x %d repeats, %d pipelines: %.1f pairs/s (%.3f ms per pair), %d PbMap failures\n", pairs,
                repeats, sp.pipelines, pairs * repeats / dt, dt / (pairs * repeats) * 1e3, failed);
    std::printf("end pose:");
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) std::printf(" %.6f", T(r, c));
    std::printf("\n");
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 3 && std::string(argv[1]) == "--throughput") {
        try {
            return throughput(std::atoi(argv[2]), argc > 3 ? std::atoi(argv[3]) : 3, argc > 4 ? std::atoi(argv[4]) : 0);
        } catch (const std::exception& e) {
            std::fprintf(stderr, "error: %s\n", e.what());
            return 2;
        }
    }
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <dir> [first] [step] [calib_dir] | --synthetic <n_frames>\n", argv[0]);
        return 1;
    }
    const bool synthetic = std::string(argv[1]) == "--synthetic";
    const int n_synth = synthetic && argc > 2 ? std::atoi(argv[2]) : 32;
    const bool skip = !synthetic || (argc > 3 && std::atoi(argv[3]) != 0);
    const std::string dir = argv[1];
    int frame = !synthetic && argc > 2 ? std::atoi(argv[2]) : 1;
    const int step = !synthetic && argc > 3 ? std::atoi(argv[3]) : 1;
    const std::string calib_dir = !synthetic && argc > 4 ? argv[4] : std::string(RGBD360_DATA_DIR) + "/calib";
    try {
        r360::Context ctx(0);
        r360::Calib360 calib(ctx, synthetic ? 480 : 240, synthetic ? 640 : 320);
        calib.loadExtrinsicCalibration(calib_dir + "/Extrinsics");
        if (!synthetic) calib.loadIntrinsicCalibration(calib_dir + "/Intrinsics");
        r360_icp_params icp;
        r360_icp_default_params(&icp);
        icp.n_pyr = 5;                                       // OdometryRGBD360.cpp:92-95
        icp.std_dev_photo = 3.0f / 255;
        const uint32_t seed = 360u << 16;
        std::vector<uint8_t> bgr;
        std::vector<uint16_t> depth;
        auto load = [&](r360::Frame360& f, int idx) -> bool {
            if (synthetic) {
                if (idx >= n_synth) return false;
                float P[16];
                r360_synth_path_pose(seed, idx, P);
                bgr.resize(size_t(8) * 480 * 640 * 3);
                depth.resize(size_t(8) * 480 * 640);
                r360::check(r360_synth_frame(calib.get(), seed, P, bgr.data(), depth.data()), "synth_frame");
                f.upload(bgr.data(), depth.data());
                return true;
            }
            const std::string path = dir + "/sphere_images_" + std::to_string(idx) + ".bin";
            if (!fexists(path)) return false;
            f.loadFrame(path);
            return true;
        };
        auto build = [&](r360::Frame360& f) {
            f.getPlanes();
            f.stitchSphericalImage();
        };
        std::unique_ptr<r360::Frame360> f1(new r360::Frame360(&calib));
        if (!load(*f1, frame)) { std::fprintf(stderr, "no first frame\n"); return 3; }
        build(*f1);
        r360::RegisterRGBD360 registerer(ctx, std::string(RGBD360_DATA_DIR) + "/config_files/configLocaliser_sphericalOdometry.ini");
        r360::Matrix4f currentPose, prevRel;
        int n_kf = 1;
        for (int idx = frame + step;; idx += step) {
            std::unique_ptr<r360::Frame360> f2(new r360::Frame360(&calib));
            if (!load(*f2, idx)) break;
            build(*f2);
            r360::Matrix4f rigidTransf;
            const bool pbmap_ok = registerer.Register(f1.get(), f2.get(), icp, rigidTransf, prevRel, 25,
                                                      r360::RegisterRGBD360::PLANAR_3DoF);
            const float dist = std::sqrt(rigidTransf(0, 3) * rigidTransf(0, 3) + rigidTransf(1, 3) * rigidTransf(1, 3) +
                                         rigidTransf(2, 3) * rigidTransf(2, 3));
            std::printf("frame %d: PbMap %s, dist %.3f\n", idx, pbmap_ok ? "ok" : "failed (dense from prior)", dist);
            if (dist < 0.4f && skip) continue;                // skip frames too close to the keyframe (:230-238)
            currentPose = currentPose * rigidTransf;          // :257
            prevRel = rigidTransf;
            if (pbmap_ok) {                                   // frame360_1 = frame360_2 only if bGoodRegistration
                f1 = std::move(f2);
                ++n_kf;
            }
            std::printf("  pose %d:", idx);
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 4; ++c) std::printf(" %.6f", currentPose(r, c));
            std::printf("\n");
        }
        std::printf("%d keyframes\n", n_kf);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 2;
    }
    return 0;
}
