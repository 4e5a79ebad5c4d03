// SphereGraphTracking — the front end of the reference's SLAM/SphereGraphSLAM.cpp over the MI355X library:
// each new Frame360 is registered (PbMap, PLANAR_ODOMETRY_3DoF) against up to numCheckRegistration = 5 of the
// newest keyframes, newest first, and becomes a keyframe with currentPose *= getPose() when one registration
// succeeds (:169-231).  The candidates of a frame are registered at once on a BatchRegistration; the winner is
// the one the sequential loop would pick.  Every `lc_every` keyframes, the newest keyframe is checked against
// the older keyframes closer than 5 m (LoopClosure360.h:291-298) in one batched call with the PbMap gate and
// alignFrames360 refinement.  Graph optimisation, submaps and the viewer are out of scope.
//   usage: SphereGraphTracking <dir with sphere_images_<n>.bin> [first] [step] [calib_dir]
//          SphereGraphTracking --synthetic <n_frames>        (procedural room, 8 x 480x640, no I/O)
#include <rgbd360/rgbd360.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <sys/stat.h>
#include <vector>

static bool fexists(const std::string& p) { struct stat st; return stat(p.c_str(), &st) == 0; }

static r360::Matrix4f inverse_rigid(const r360::Matrix4f& T) {
    r360::Matrix4f o;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) o(r, c) = T(c, r);
    for (int r = 0; r < 3; ++r) o(r, 3) = -(o(r, 0) * T(0, 3) + o(r, 1) * T(1, 3) + o(r, 2) * T(2, 3));
    return o;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <dir> [first] [step] [calib_dir] | --synthetic <n_frames>\n", argv[0]);
        return 1;
    }
    const bool synthetic = std::string(argv[1]) == "--synthetic";
    const int n_synth = synthetic && argc > 2 ? std::atoi(argv[2]) : 16;
    const std::string dir = argv[1];
    const int first = !synthetic && argc > 2 ? std::atoi(argv[2]) : (synthetic ? 0 : 1);
    const int step = !synthetic && argc > 3 ? std::atoi(argv[3]) : 1;
    const std::string calib_dir = !synthetic && argc > 4 ? argv[4] : std::string(RGBD360_DATA_DIR) + "/calib";
    const int numCheckRegistration = 5, noAssoc_threshold = 40, lc_every = 4;   // SphereGraphSLAM.cpp:99-100
    try {
        r360::Context ctx(0);
        r360::Calib360 calib(ctx, synthetic ? 480 : 240, synthetic ? 640 : 320);
        calib.loadExtrinsicCalibration(calib_dir + "/Extrinsics");
        if (!synthetic) calib.loadIntrinsicCalibration(calib_dir + "/Intrinsics");
        r360_icp_params icp;
        r360_icp_default_params(&icp);
        icp.n_pyr = 5;
        icp.std_dev_photo = 3.0f / 255;
        r360::BatchRegistration batch(0, 8);
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
        std::vector<std::unique_ptr<r360::Frame360> > kfs;
        std::vector<r360::Matrix4f> poses;
        int n_lc = 0;
        for (int idx = first;; idx += step) {
            std::unique_ptr<r360::Frame360> f(new r360::Frame360(&calib));
            if (!load(*f, idx)) break;
            f->getPlanes();
            f->stitchSphericalImage();
            if (kfs.empty()) {
                kfs.push_back(std::move(f));
                poses.push_back(r360::Matrix4f::Identity());
                continue;
            }
            std::vector<r360::Frame360*> kf;
            for (auto& k : kfs) kf.push_back(k.get());
            r360_pair_result win;
            const int j = batch.track(kf, f.get(), &win, numCheckRegistration, noAssoc_threshold);
            if (j < 0) {
                std::printf("frame %d: No registration available\n", idx);
                continue;
            }
            r360::Matrix4f rel;
            std::memcpy(rel.data(), win.pbmap_pose, sizeof win.pbmap_pose);
            poses.push_back(poses[j] * rel);
            std::printf("frame %d: Good TRACKING with keyframe %d, %d matches, SSO %.3f\n", idx, j, win.n_match,
                        win.sso_pbmap);
            kfs.push_back(std::move(f));
            if (int(kfs.size()) % lc_every == 0) {       // loop-closure candidates of the newest keyframe
                std::vector<std::pair<r360::Frame360*, r360::Frame360*> > pairs;
                std::vector<int> ids;
                const int nk = int(kfs.size()) - 1;
                for (int k = 0; k + numCheckRegistration < nk; ++k) {
                    const r360::Matrix4f rp = inverse_rigid(poses[k]) * poses[nk];
                    if (std::sqrt(rp(0, 3) * rp(0, 3) + rp(1, 3) * rp(1, 3) + rp(2, 3) * rp(2, 3)) < 5.f) {
                        pairs.push_back({kfs[k].get(), kfs[nk].get()});
                        ids.push_back(k);
                    }
                }
                const auto res = batch.loopClosures(pairs, icp);
                for (size_t i = 0; i < res.size(); ++i)
                    if (res[i].dense_rc >= 0) {
                        ++n_lc;
                        std::printf("  loop closure %d - %d: SSO %.3f\n", ids[i], nk, res[i].stats.sso);
                    }
            }
        }
        std::printf("%zu keyframes, %d loop-closure edges\n", kfs.size(), n_lc);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 2;
    }
    return 0;
}
