// KFsphereTracking — the tracking front end of the reference's SLAM/KFsphere_SLAM.cpp written against the
// façade (include/rgbd360/rgbd360.h) with the reference's own calls:
//   RegisterPbMap(kf, frame, 25, PLANAR_3DoF), getPose, calcEntropy, getMatchedPlanes, getAreaMatched,
//   trackingScore (:314-317, RegisterRGBD360.h:526); RegisterPhotoICP setNumPyr / useSaliency /
//   setVisualization / setGrayVariance (:279-283), setTargetFrame(kf->sphereRGB, kf->sphereDepth),
//   setSourceFrame(frame->sphereRGB, frame->sphereDepth) (:370-371), alignFrames360(init, PHOTO_DEPTH, occ)
//   (:373), getOptimalPose, avPhotoResidual / avDepthResidual (:379-388), getHessian, SSO (:401-402).
// A frame becomes a keyframe when the dense registration moved more than 0.4 m from the current keyframe or
// its depth residual exceeds selectKF_ICPdist (the reference's test :388); the trajectory is the keyframe
// chain.  Graph optimisation, loop closure and the viewer are out of scope.
// avDepthResidual is assigned only by the occlusion variants (RegisterPhotoICP.h:3360-3362, :3852-3853);
// with occlusion 0 it keeps its previous value (NaN here, uninitialised in the reference), so the residual
// test applies only with occlusion 1 / 2.
//   usage: KFsphereTracking --synthetic <n_frames> [occlusion]      (procedural room, 8 x 480x640)
//          KFsphereTracking <dir with sphere_images_<n>.bin> [first] [step] [calib_dir] [occlusion]
#include <rgbd360/rgbd360.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <sys/stat.h>
#include <vector>

static bool fexists(const std::string& p) { struct stat st; return stat(p.c_str(), &st) == 0; }

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s --synthetic <n_frames> [occlusion] | <dir> [first] [step] [calib_dir] [occlusion]\n",
                     argv[0]);
        return 1;
    }
    const bool synthetic = std::string(argv[1]) == "--synthetic";
    const int n_synth = synthetic && argc > 2 ? std::atoi(argv[2]) : 8;
    const std::string dir = argv[1];
    const int first = !synthetic && argc > 2 ? std::atoi(argv[2]) : (synthetic ? 0 : 1);
    const int step = !synthetic && argc > 3 ? std::atoi(argv[3]) : 1;
    const std::string calib_dir = !synthetic && argc > 4 ? argv[4] : std::string(RGBD360_DATA_DIR) + "/calib";
    const int occlusion = synthetic ? (argc > 3 ? std::atoi(argv[3]) : 0) : (argc > 5 ? std::atoi(argv[5]) : 0);
    const float selectKF_ICPdist = 0.9f;                 // KFsphere_SLAM.cpp:388 threshold (selectKF_ICPdist)
    try {
        r360::Context ctx(0);
        r360::Calib360 calib(ctx, synthetic ? 480 : 240, synthetic ? 640 : 320);
        calib.loadExtrinsicCalibration(calib_dir + "/Extrinsics");
        if (!synthetic) calib.loadIntrinsicCalibration(calib_dir + "/Intrinsics");
        r360::RegisterRGBD360 registerer(ctx, std::string(RGBD360_DATA_DIR) + "/config_files/configLocaliser_sphericalOdometry.ini");
        r360::RegisterPhotoICP align360(ctx);            // :279-283
        align360.setNumPyr(5);
        align360.useSaliency(false);
        align360.setVisualization(false);
        align360.setGrayVariance(3.f / 255);
        // rotOffset (angleOffset 157.5 deg about x, float angle, double PI): the sphere vs the rig frame
        const float angleOffset = 157.5f;
        r360::Matrix4f rotOffset, rotOffsetInv;
        rotOffset(1, 1) = rotOffset(2, 2) = std::cos(angleOffset * 3.14159265359 / 180);
        rotOffset(1, 2) = std::sin(angleOffset * 3.14159265359 / 180);
        rotOffset(2, 1) = -rotOffset(1, 2);
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) rotOffsetInv(r, c) = rotOffset(c, r);

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
        std::vector<r360::Matrix4f> kfPose;
        kfs.emplace_back(new r360::Frame360(&calib));
        if (!load(*kfs.back(), first)) { std::fprintf(stderr, "no first frame\n"); return 3; }
        kfs.back()->getPlanes();
        kfs.back()->stitchSphericalImage();
        kfPose.push_back(r360::Matrix4f::Identity());
        r360::Matrix4f rigidTransf_dense_ref = r360::Matrix4f::Identity();   // sphere-frame init (:372-375)
        for (int idx = first + step;; idx += step) {
            std::unique_ptr<r360::Frame360> frame(new r360::Frame360(&calib));
            if (!load(*frame, idx)) break;
            frame->getPlanes();
            frame->stitchSphericalImage();
            r360::Frame360* kf = kfs.back().get();
            const bool bGoodTracking = registerer.RegisterPbMap(kf, frame.get(), 25, r360::RegisterRGBD360::PLANAR_3DoF);
            const r360::Matrix4f trackedPosePbMap = registerer.getPose();
            float score = 0.f;
            const int quality = bGoodTracking ? registerer.trackingScore(score) : 2;
            std::printf("frame %d: PbMap %s entropy %.4f matches %zu area %.3f score %.3f quality %d\n", idx,
                        bGoodTracking ? "ok" : "failed", bGoodTracking ? registerer.calcEntropy() : 0.f,
                        registerer.getMatchedPlanes().size(), registerer.getAreaMatched(), score, quality);
            if (bGoodTracking) rigidTransf_dense_ref = rotOffset * trackedPosePbMap * rotOffsetInv;
            align360.setTargetFrame(kf->sphereRGB, kf->sphereDepth);            // :370-371
            align360.setSourceFrame(frame->sphereRGB, frame->sphereDepth);
            const bool ok = align360.alignFrames360(rigidTransf_dense_ref, r360::RegisterPhotoICP::PHOTO_DEPTH, occlusion);
            rigidTransf_dense_ref = align360.getOptimalPose();
            const r360::Matrix4f rigidTransf_dense = rotOffsetInv * rigidTransf_dense_ref * rotOffset;
            const r360::Matrix6f hessian = align360.getHessian();
            const float dist = std::sqrt(rigidTransf_dense(0, 3) * rigidTransf_dense(0, 3) +
                                         rigidTransf_dense(1, 3) * rigidTransf_dense(1, 3) +
                                         rigidTransf_dense(2, 3) * rigidTransf_dense(2, 3));
            std::printf("  dense %s: dist %.3f Residuals: %.5f %.5f SSO %.3f H00 %.3g\n", ok ? "ok" : "ILL-POSED", dist,
                        align360.avPhotoResidual, align360.avDepthResidual, align360.SSO, hessian(0, 0));
            const bool far = dist > 0.4f || (occlusion && !(align360.avDepthResidual < selectKF_ICPdist));
            if (far) {                                   // a new keyframe: its pose is the chain of dense poses
                kfPose.push_back(kfPose.back() * rigidTransf_dense);
                kfs.push_back(std::move(frame));
                rigidTransf_dense_ref = r360::Matrix4f::Identity();
                const r360::Matrix4f& P = kfPose.back();
                std::printf("  keyframe %d t = (%.4f %.4f %.4f)\n", idx, P(0, 3), P(1, 3), P(2, 3));
            }
        }
        std::printf("%zu keyframes\n", kfs.size());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 2;
    }
    return 0;
}
