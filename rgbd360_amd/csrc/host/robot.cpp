// robot.cpp — host side of SURVEY §8(a) A19, RegisterRGBD360::RegisterDensePhotoICP
// (include/RegisterRGBD360.h:344-520): the 8 sensors' pinhole images of frame2 (source) aligned to
// frame1's (target) with the sensor Jacobians expressed in the rig frame
// (calcPhotoICPError_robot / calcHessianGradient_robot, RegisterPhotoICP.h:4905-5407).
// Every (level, sensor) job is evaluated at the initial pose in one launch, then a one-wave kernel
// replays the level loop (robot_kernels.hip explains why the reference never moves the pose).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "../r360_internal.h"


namespace {

void matmul4(const float* A, const float* B, float* Cm) {   // Eigen Matrix4f product order (col-major)
    float out[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) {
            float s = A[r] * B[c * 4];
            for (int k = 1; k < 4; ++k) s += A[k * 4 + r] * B[c * 4 + k];
            out[c * 4 + r] = s;
        }
    memcpy(Cm, out, sizeof(out));
}

int ensure_robot_buffers(r360_ctx* ctx) {
    if (ctx->d_rob_jobs) return 0;
    const int NJ = R360_ROBOT_MAX_JOBS;
    R360_HIP(hipMalloc(&ctx->d_rob_jobs, sizeof(RobotJob) * NJ));
    R360_HIP(hipHostMalloc(&ctx->h_rob_jobs, sizeof(RobotJob) * NJ, hipHostMallocDefault));
    R360_HIP(hipMalloc(&ctx->d_rob_partials, sizeof(double) * 32 * R360_ROBOT_MAX_BLOCKS * NJ));
    R360_HIP(hipMalloc(&ctx->d_rob_sums, sizeof(double) * 32 * NJ));
    R360_HIP(hipHostMalloc(&ctx->h_rob_sums, sizeof(double) * 32 * NJ, hipHostMallocDefault));
    R360_HIP(hipMalloc(&ctx->d_rob_tickets, sizeof(unsigned) * NJ));
    R360_HIP(hipMemsetAsync(ctx->d_rob_tickets, 0, sizeof(unsigned) * NJ, ctx->stream));   // ordered before its kernels
    R360_HIP(hipMalloc(&ctx->d_rob_out, sizeof(RobotOut)));
    R360_HIP(hipHostMalloc(&ctx->h_rob_out, sizeof(RobotOut), hipHostMallocDefault));
    return 0;
}

int check_pair(r360_ctx* ctx, r360_frame* f1, r360_frame* f2, int method, const r360_icp_params* p) {
    CHECK_ARG(ctx && f1 && f2 && p, "null arg");
    CHECK_ARG(f1->rows == f2->rows && f1->cols == f2->cols, "frame size mismatch");
    CHECK_ARG((f1->built & R360_BUILD_SENSOR_PYRAMID) && (f2->built & R360_BUILD_SENSOR_PYRAMID),
              "frames need R360_BUILD_SENSOR_PYRAMID (setSourceFrame/setTargetFrame of the sensor images)");
    CHECK_ARG(f1->calib, "frame1 has no calibration");
    CHECK_ARG(p->n_pyr >= 1 && p->n_pyr <= f2->n_slevels && p->n_pyr <= 8, "n_pyr exceeds the sensor pyramid depth");
    CHECK_ARG(p->min_depth == 0.3f && p->max_depth == 6.0f,
              "non-default min/max depth changes the depth pyramid: not supported in this version");
    CHECK_ARG(method >= 0 && method <= 2, "invalid method");
    return 0;
}

// The jobs of `levels` (l * 8 + k order) at `pose`.  camIntrinsicMat is RegisterDensePhotoICP's own
// (RegisterRGBD360.h:357-365): focal 525 * (cols / 640.0), centre (cols/2 - 0.5, rows/2 - 0.5).
int enqueue_jobs(r360_ctx* ctx, r360_frame* f1, r360_frame* f2, int l_lo, int l_hi, const float pose[16], int method,
                 const r360_icp_params* p, int finalize_levels) {
    const float img_width = (float)f1->cols, img_height = (float)f1->rows;
    const float res_factor_VGA = (float)(img_width / 640.0);
    const float focal = 525 * res_factor_VGA;
    const float K00 = focal, K11 = focal;
    const float K02 = (float)(img_width / 2 - 0.5), K12 = (float)(img_height / 2 - 0.5);
    RobotGrid grid;
    memset(&grid, 0, sizeof(grid));
    int nj = 0, blocks = 0;
    for (int l = l_lo; l <= l_hi; ++l) {
        const LevelBufs& Ls = f2->sp[l];
        const LevelBufs& Lt = f1->sp[l];
        // calcPhotoICPError_robot (:4917-4924): float scaleFactor and intrinsics, float inv = 1./f
        const float scf = (float)(1.0 / pow(2, l));
        // calcHessianGradient_robot (:5093-5099): double scaleFactor and intrinsics
        const double scd = 1.0 / pow(2, l);
        const int npx = Ls.rows * Ls.cols;
        int nb = (npx + TPB_ROBOT * 4 - 1) / (TPB_ROBOT * 4);
        if (nb < 1) nb = 1;
        if (nb > R360_ROBOT_MAX_BLOCKS) nb = R360_ROBOT_MAX_BLOCKS;
        for (int k = 0; k < 8; ++k) {
            RobotJob& J = ctx->h_rob_jobs[nj];
            const long off = (long)k * npx;
            J.src = Ls.p0 + off; J.trg = Lt.p0 + off; J.tg = Lt.tg + off;
            J.rows = Ls.rows; J.cols = Ls.cols;
            J.fx = K00 * scf; J.fy = K11 * scf; J.ox = K02 * scf; J.oy = K12 * scf;
            J.inv_fx = (float)(1. / J.fx); J.inv_fy = (float)(1. / J.fy);
            J.fxd = K00 * scd; J.fyd = K11 * scd; J.oxd = K02 * scd; J.oyd = K12 * scd;
            J.inv_fxd = 1. / J.fxd; J.inv_fyd = 1. / J.fyd;
            // poseCamRobot = calib->Rt_[k], its inverse = Rt_[k].inverse() = calib->Rt_inv[k]
            memcpy(J.Rt, f1->calib->rt[k], sizeof(J.Rt));
            memcpy(J.Rti, f1->calib->rt_inv[k], sizeof(J.Rti));
            memcpy(J.P, pose, sizeof(J.P));
            float tmp[16];
            matmul4(J.Rti, J.P, tmp);              // relPoseCam = poseCamRobot_inv * poseGuess * poseCamRobot
            matmul4(tmp, J.Rt, J.Mrel);
            grid.block0[nj] = blocks;
            blocks += nb;
            ++nj;
        }
    }
    grid.block0[nj] = blocks;
    grid.njobs = nj;
    IcpConst C;
    memset(&C, 0, sizeof(C));
    C.min_d = p->min_depth; C.max_d = p->max_depth;
    C.sd_photo = p->std_dev_photo; C.sd_depth = p->std_dev_depth;
    C.thr_int = p->thres_sal_int; C.thr_depth = p->thres_sal_depth;
    C.sd_photo_inv_d = 1. / p->std_dev_photo;      // double stdDevPhoto_inv (:4929, :5107)
    R360_HIP(hipMemcpyAsync(ctx->d_rob_jobs, ctx->h_rob_jobs, sizeof(RobotJob) * nj, hipMemcpyHostToDevice,
                            ctx->stream));
    return launch_robot(ctx, ctx->d_rob_jobs, grid, method, C, finalize_levels);
}

}  // namespace

extern "C" int r360_register_dense(r360_ctx* ctx, r360_frame* frame1, r360_frame* frame2, const float pose_estim[16],
                                   int method, int mode, const r360_icp_params* p_in, float pose_out[16],
                                   float info_out[36], r360_dense_stats* st) {
    if (ctx && bind_device(ctx->device)) return -1;
    (void)mode;   // registMode is accepted and unused by the reference (RegisterRGBD360.h:344-520)
    r360_icp_params pd;
    r360_icp_default_params(&pd);                  // the RegisterPhotoICP() the function constructs
    const r360_icp_params* p = p_in ? p_in : &pd;
    if (int rc = check_pair(ctx, frame1, frame2, method, p)) return rc;
    CHECK_ARG(pose_estim, "null pose");
    if (ensure_robot_buffers(ctx)) return -1;
    const int nL = p->n_pyr;
    if (enqueue_jobs(ctx, frame1, frame2, 0, nL - 1, pose_estim, method, p, nL)) return -1;
    R360_HIP(hipMemcpyAsync(ctx->h_rob_out, ctx->d_rob_out, sizeof(RobotOut), hipMemcpyDeviceToHost, ctx->stream));
    if (ctx_wait(ctx)) return -1;
    const RobotOut& o = *ctx->h_rob_out;
    if (st) {
        memset(st, 0, sizeof(*st));
        for (int l = 0; l < nL; ++l) {
            st->error[l] = o.error[l]; st->ran[l] = o.ran[l];
            st->n_visible[l] = o.n_visible[l]; st->n_error[l] = o.n_error[l];
        }
        st->illposed_level = o.illposed_level;
        st->levels = nL;
        st->info_set = o.any;
        memcpy(st->gradient, o.grad, sizeof(st->gradient));
    }
    // rigidTransf = pose_estim on both returns (:430, :512); informationM = Hessian only on success
    if (pose_out) memcpy(pose_out, pose_estim, sizeof(float) * 16);
    if (!o.ok) return 0;
    if (info_out) {
        if (o.any) memcpy(info_out, o.info, sizeof(float) * 36);
        else memset(info_out, 0, sizeof(float) * 36);   // no level ran: the reference's Hessian is uninitialised
    }
    return 1;
}

extern "C" int r360_dense_robot_eval(r360_ctx* ctx, r360_frame* frame1, r360_frame* frame2, int level,
                                     const float pose[16], int method, const r360_icp_params* p_in, double err[16],
                                     double H[8 * 36], double g[8 * 6], int counts[8 * 3]) {
    r360_icp_params pd;
    r360_icp_default_params(&pd);
    const r360_icp_params* p = p_in ? p_in : &pd;
    if (int rc = check_pair(ctx, frame1, frame2, method, p)) return rc;
    CHECK_ARG(level >= 0 && level < frame2->n_slevels && pose, "level out of range / null pose");
    if (ensure_robot_buffers(ctx)) return -1;
    if (enqueue_jobs(ctx, frame1, frame2, level, level, pose, method, p, 0)) return -1;
    R360_HIP(hipMemcpyAsync(ctx->h_rob_sums, ctx->d_rob_sums, sizeof(double) * 32 * 8, hipMemcpyDeviceToHost,
                            ctx->stream));
    if (ctx_wait(ctx)) return -1;
    for (int k = 0; k < 8; ++k) {
        const double* s = ctx->h_rob_sums + k * 32;
        if (err) { err[2 * k] = s[R360_SUM_ERR2]; err[2 * k + 1] = s[R360_SUM_ERR2D]; }
        int q = 0;
        for (int u = 0; u < 6; ++u)
            for (int v = u; v < 6; ++v) {
                if (H) H[k * 36 + u * 6 + v] = H[k * 36 + v * 6 + u] = s[q];
                ++q;
            }
        for (int u = 0; u < 6; ++u) if (g) g[k * 6 + u] = s[21 + u];
        if (counts) {
            counts[3 * k] = (int)s[R360_SUM_NVALID];
            counts[3 * k + 1] = (int)s[R360_SUM_NDEPTH];
            counts[3 * k + 2] = (int)s[R360_SUM_NVIS];
        }
    }
    return 0;
}
