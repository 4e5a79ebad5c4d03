// pinhole.cpp — host side of §8(f) rank 3, RegisterPhotoICP's per-sensor pinhole alignFrames
// (include/RegisterPhotoICP.h:4254-4512) over the per-sensor pyramids of two Frame360s
// (R360_BUILD_SENSOR_PYRAMID).  Up to 8 alignments (one per listed sensor) are enqueued as one batched
// pass sequence; every pass after a job has converged returns at its first instruction.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../r360_internal.h"


namespace {

int ensure_pin_buffers(r360_ctx* ctx) {
    if (ctx->d_pin_state) return 0;
    R360_HIP(hipMalloc(&ctx->d_pin_state, sizeof(IcpState) * 8));
    R360_HIP(hipMalloc(&ctx->d_pin_partials, sizeof(double) * 32 * R360_PIN_MAX_BLOCKS * 8));
    R360_HIP(hipHostMalloc(&ctx->h_pin_state, sizeof(IcpState) * 8, hipHostMallocDefault));
    return 0;
}

// IcpConst of a pinhole pass: the RegisterPhotoICP members alignFrames reads (depth range, std devs,
// saliency thresholds); its LM constants live in the kernel (pinhole_kernels.hip)
IcpConst pin_const(const r360_icp_params* p, int level) {
    IcpConst C;
    memset(&C, 0, sizeof(C));
    C.min_d = p->min_depth; C.max_d = p->max_depth;
    C.sd_photo = p->std_dev_photo; C.sd_depth = p->std_dev_depth;
    C.thr_int = p->thres_sal_int; C.thr_depth = p->thres_sal_depth;
    C.sd_photo_inv_f = (float)(1. / p->std_dev_photo);
    C.sd_photo_inv_d = 1. / p->std_dev_photo;
    C.max_iters = 10;
    C.level = level;
    return C;
}

int check_pin_pair(r360_ctx* ctx, r360_frame* trg, r360_frame* src, const r360_icp_params* p) {
    CHECK_ARG(ctx && trg && src && p, "null arg");
    CHECK_ARG(trg->rows == src->rows && trg->cols == src->cols, "frame size mismatch");
    CHECK_ARG((trg->built & R360_BUILD_SENSOR_PYRAMID) && (src->built & R360_BUILD_SENSOR_PYRAMID),
              "frames need R360_BUILD_SENSOR_PYRAMID (setSourceFrame/setTargetFrame of the sensor images)");
    CHECK_ARG(p->n_pyr >= 1 && p->n_pyr <= src->n_slevels, "n_pyr exceeds the sensor pyramid depth");
    CHECK_ARG(p->min_depth == 0.3f && p->max_depth == 6.0f,
              "non-default min/max depth changes the depth pyramid: not supported in this version");
    return 0;
}

// cameraMatrix as setCameraMatrix sets it; NULL = the calibration's (f = 525*cols/640, c = (cols/2-0.5,
// rows/2-0.5), the Methods harness's own values, MethodsRegisterRGBD360.cpp:323-330)
void intrinsics(const r360_frame* f, const float* K_in, float K[4]) {
    if (K_in) { memcpy(K, K_in, sizeof(float) * 4); return; }
    const float* C = f->calib->K;
    K[0] = C[0]; K[1] = C[4]; K[2] = C[6]; K[3] = C[7];
}

}  // namespace

extern "C" int r360_align_pinhole_async(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int n, const int* sensors,
                                        const float* init, int method, const float* K_in, const r360_icp_params* p) {
    if (ctx && bind_device(ctx->device)) return -1;
    if (int rc = check_pin_pair(ctx, trg, src, p)) return rc;
    CHECK_ARG(n >= 1 && n <= 8 && sensors && init, "1..8 jobs with sensors and init poses");
    CHECK_ARG(method >= 0 && method <= 2, "invalid method");
    for (int j = 0; j < n; ++j) CHECK_ARG(sensors[j] >= 0 && sensors[j] < 8, "sensor out of range");
    if (ensure_pin_buffers(ctx)) return -1;
    PinJobs J;
    memset(&J, 0, sizeof(J));
    J.n = n;
    IcpState* h = ctx->h_pin_state;
    memset(h, 0, sizeof(IcpState) * 8);
    for (int j = 0; j < n; ++j) {
        J.sensor[j] = sensors[j];
        memcpy(h[j].pose, init + 16 * j, sizeof(float) * 16);
        memcpy(h[j].cand, init + 16 * j, sizeof(float) * 16);
    }
    float K[4];
    intrinsics(src, K_in, K);
    R360_HIP(hipMemcpyAsync(ctx->d_pin_state, h, sizeof(IcpState) * n, hipMemcpyHostToDevice, ctx->stream));
    // per level: the error + H at pose_estim, then at most 2 candidate evaluations per iteration
    // (the undamped step and the LM retry, :4324-4412)
    const int passes = 1 + 2 * 10;
    for (int l = p->n_pyr - 1; l >= 0; --l) {
        const IcpConst C = pin_const(p, l);
        for (int k = 0; k < passes; ++k)
            if (launch_pin_level(ctx, trg, src, l, method, C, K, J, k == 0, 0)) return -1;
    }
    ctx->pin_pending = n;
    return 0;
}

extern "C" int r360_align_pinhole_result(r360_ctx* ctx, float* poses, float* H, float* g, r360_icp_stats* st) {
    CHECK_ARG(ctx && ctx->pin_pending, "no pinhole alignment pending");
    const int n = ctx->pin_pending;
    IcpState* h = ctx->h_pin_state;
    R360_HIP(hipMemcpyAsync(h, ctx->d_pin_state, sizeof(IcpState) * n, hipMemcpyDeviceToHost, ctx->stream));
    if (ctx_wait(ctx)) return -1;
    ctx->pin_pending = 0;
    int ill = 0;
    for (int j = 0; j < n; ++j) {
        if (poses) memcpy(poses + 16 * j, h[j].pose, sizeof(float) * 16);
        if (H) memcpy(H + 36 * j, h[j].Hout, sizeof(float) * 36);
        if (g) memcpy(g + 6 * j, h[j].gout, sizeof(float) * 6);
        if (st) {
            r360_icp_stats& s = st[j];
            memset(&s, 0, sizeof(s));
            for (int l = 0; l < 8; ++l) { s.iters[l] = h[j].iters[l]; s.evals[l] = h[j].evals_l[l]; }
            s.illposed = h[j].illposed;
            s.error = h[j].error;
            s.passes = h[j].passes;
            // alignFrames restores the copies of the last loop iteration's start (:4507-4509); an ILL-POSED
            // return skips that, leaving the last evaluation's values (equal to those copies)
            const bool t = (h[j].av_set & 12) != 0;
            s.av_photo_residual = (t && !h[j].illposed) ? h[j].av_photo_t : h[j].av_photo;
            s.av_depth_residual = (t && !h[j].illposed) ? h[j].av_depth_t : h[j].av_depth;
            s.av_residual = (t && !h[j].illposed) ? h[j].av_res_t : h[j].av_res;
            s.residuals_set = (t || h[j].illposed) ? 3 : 0;
        }
        ill += h[j].illposed;
    }
    return ill;
}

extern "C" int r360_align_pinhole(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int sensor, const float init[16],
                                  int method, const float* K, const r360_icp_params* p, float pose_out[16],
                                  float H_out[36], float g_out[6], r360_icp_stats* st) {
    if (int rc = r360_align_pinhole_async(ctx, trg, src, 1, &sensor, init, method, K, p)) return rc;
    return r360_align_pinhole_result(ctx, pose_out, H_out, g_out, st) ? 1 : 0;
}

// One eval-mode pass: errorPhotoICP's sums and calcHessGrad's H / g at `pose`.
extern "C" int r360_pinhole_eval(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int sensor, int level,
                                 const float pose[16], int method, const float* K_in, const r360_icp_params* p,
                                 double H[36], double g[6], double* error, double res[2], int counts[3]) {
    if (int rc = check_pin_pair(ctx, trg, src, p)) return rc;
    CHECK_ARG(sensor >= 0 && sensor < 8, "sensor out of range");
    CHECK_ARG(level >= 0 && level < src->n_slevels, "level out of range");
    CHECK_ARG(method >= 0 && method <= 2 && pose, "invalid method / pose");
    if (ensure_pin_buffers(ctx)) return -1;
    PinJobs J;
    memset(&J, 0, sizeof(J));
    J.n = 1;
    J.sensor[0] = sensor;
    IcpState* h = ctx->h_pin_state;
    memset(h, 0, sizeof(IcpState));
    memcpy(h->pose, pose, sizeof(float) * 16);
    memcpy(h->cand, pose, sizeof(float) * 16);
    float K[4];
    intrinsics(src, K_in, K);
    R360_HIP(hipMemcpyAsync(ctx->d_pin_state, h, sizeof(IcpState), hipMemcpyHostToDevice, ctx->stream));
    if (launch_pin_level(ctx, trg, src, level, method, pin_const(p, level), K, J, 0, 1)) return -1;
    R360_HIP(hipMemcpyAsync(h, ctx->d_pin_state, sizeof(IcpState), hipMemcpyDeviceToHost, ctx->stream));
    if (ctx_wait(ctx)) return -1;
    const double* s = h->sums;
    int k = 0;
    for (int u = 0; u < 6; ++u)
        for (int v = u; v < 6; ++v) { if (H) H[u * 6 + v] = H[v * 6 + u] = s[k]; ++k; }
    for (int u = 0; u < 6; ++u) if (g) g[u] = s[21 + u];
    const double nD = s[R360_SUM_NDEPTH];
    if (error) *error = sqrt(s[R360_SUM_ERR2] / nD) + sqrt(s[R360_SUM_ERR2D] / nD);
    if (res) { res[0] = s[R360_SUM_ERR2]; res[1] = s[R360_SUM_ERR2D]; }
    if (counts) { counts[0] = (int)s[R360_SUM_NVALID]; counts[1] = (int)nD; counts[2] = (int)s[R360_SUM_NVIS]; }
    return 0;
}
