// robot_kernels.hip — SURVEY §8(a) A19: RegisterRGBD360::RegisterDensePhotoICP on gfx950, the per-sensor
// pinhole direct alignment of two Frame360s expressed in the rig ("robot") frame.
//
//   RegisterDensePhotoICP       include/RegisterRGBD360.h:344-520   (8 sensors summed, LM per level)
//   calcPhotoICPError_robot     include/RegisterPhotoICP.h:4905-5076 (all-pixel branch :5004-5072)
//   calcHessianGradient_robot   :5083-5407                            (all-pixel branch :5261-5405)
//
// What the reference computes.  Every level evaluates the error at pose_estim, then (if it exceeds
// tol_residual = 0.1) the 8 sensors' H / g at pose_estim, the LM update and pose_estim_temp — and then
// re-evaluates the "new" error at pose_estim again (RegisterRGBD360.h:430-432 passes pose_estim, not
// pose_estim_temp).  The two evaluations are the same function of the same inputs, so diff_error = 0,
// the candidate is never accepted and the loop exits: the pose is never updated, and informationM is
// the H of the last level whose loop ran.  (The reference sums the 8 sensors' errors in an OpenMP
// reduction whose combination order is unspecified; in a deterministic order, as here and in the
// oracle, both evaluations agree bit for bit.)  All work of a call therefore happens at ONE pose, and
// every (level, sensor) job is independent: one launch evaluates all of them — error + H / g fused per
// source pixel — and a one-wave finalize kernel replays the level loop.
//
// Per source pixel the reference runs two different projections:
//   error:    float LUT ((c - ox) * z * inv_fx, float intrinsics), relPoseCam = Rt^-1 * pose * Rt
//             composed in float, 1/z and the pixel coordinates in double (:4960-4976);
//   HessGrad: double intrinsics ((c - ox) * z * inv_fx in double, stored as float), three float
//             transforms Rt, pose, Rt^-1 in turn, 1/z in double (:5266-5287).
// Both are restated expression by expression (-ffp-contract=off), so visibility, target pixels, counts
// and error terms are exact; H / g are float terms summed in double per sensor (the reference sums
// them in float in raster order, so H / g parity is within float-summation tolerance).
// jacobianRt_z (:5372-5374) is an uninitialised Eigen vector in the reference; it is taken as zero —
// the derivative of the residual as written (target depth minus the UNwarped source depth) has no
// such term.  PHOTO_CONSISTENCY, the function's default and the only method its callers use
// (MethodsRegisterRGBD360.cpp), does not read it.
#include <hip/hip_runtime.h>

#include <cmath>

#include "../r360_internal.h"

namespace {

constexpr int TPB = TPB_ROBOT;
constexpr int NW = TPB / 64;
constexpr int RG = TPB / 16;

#include "icp_common.inc"
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wunused-function"
#include "icp_la.inc"
#pragma clang diagnostic pop

struct V4 { float x, y, z, w; };

// Eigen Matrix4f * Vector4f (col-major): ((m0 x + m1 y) + m2 z) + m3 w per row
__device__ __forceinline__ V4 xform(const float* __restrict__ M, float x, float y, float z, float w) {
    V4 o;
    o.x = M[0] * x + M[4] * y; o.x = o.x + M[8] * z; o.x = o.x + M[12] * w;
    o.y = M[1] * x + M[5] * y; o.y = o.y + M[9] * z; o.y = o.y + M[13] * w;
    o.z = M[2] * x + M[6] * y; o.z = o.z + M[10] * z; o.z = o.z + M[14] * w;
    o.w = M[3] * x + M[7] * y; o.w = o.w + M[11] * z; o.w = o.w + M[15] * w;
    return o;
}

// one source pixel of job J: calcPhotoICPError_robot's terms and calcHessianGradient_robot's rows
template <int METHOD>
__device__ __forceinline__ void robot_pixel(Acc& A, const RobotJob& J, const IcpConst& C, int i, int r, int c) {
    constexpr bool photo = (METHOD == R360_PHOTO_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    constexpr bool depth = (METHOD == R360_DEPTH_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    const float2 s = J.src[i];
    const float z = s.y, gray1 = s.x;
    if (!(C.min_d < z && z < C.max_d)) return;
    const int nRows = J.rows, nCols = J.cols;

    // ---- calcPhotoICPError_robot (:5012-5068)
    {
        const float lx = (((float)c - J.ox) * z) * J.inv_fx;
        const float ly = (((float)r - J.oy) * z) * J.inv_fy;
        const V4 p = xform(J.Mrel, lx, ly, z, 1.f);
        const double inv = 1.0 / (double)p.z;
        const double tc = (double)(p.x * J.fx) * inv + (double)J.ox;
        const double tr = (double)(p.y * J.fy) * inv + (double)J.oy;
        const double rr = round(tr), cc = round(tc);
        if (rr >= 0.0 && rr < (double)nRows && cc >= 0.0 && cc < (double)nCols) {
            const int t = (int)rr * nCols + (int)cc;
            const float2 T = J.trg[t];
            A.h[27] += 1.f;
            if (photo) {
                const float photoDiff = T.x - gray1;
                const double w = (double)huberf(photoDiff, C.sd_photo) * C.sd_photo_inv_d;
                const float wE = (float)(w * (double)photoDiff);
                A.err2 += (double)(wE * wE);
            }
            if (depth && isfinite(T.y)) {
                const float depthDiff = T.y - z;
                const float sd = C.sd_depth * z;
                const float w = huberf(depthDiff, sd) / sd;
                const float wE = w * depthDiff;
                A.err2d += (double)(wE * wE);
                A.h[29] += 1.f;
            }
        }
    }

    // ---- calcHessianGradient_robot (:5266-5403)
    const float x0 = (float)((((double)c - J.oxd) * (double)z) * J.inv_fxd);
    const float y0 = (float)((((double)r - J.oyd) * (double)z) * J.inv_fyd);
    const V4 p1 = xform(J.Rt, x0, y0, z, 1.f);           // point3D_robot
    const V4 p2 = xform(J.P, p1.x, p1.y, p1.z, p1.w);    // point3D_robot2
    const V4 p3 = xform(J.Rti, p2.x, p2.y, p2.z, p2.w);  // transformedPoint3D
    const double inv = 1.0 / (double)p3.z;
    const double tc = ((double)p3.x * J.fxd) * inv + J.oxd;
    const double tr = ((double)p3.y * J.fyd) * inv + J.oyd;
    const double rr = round(tr), cc = round(tc);
    if (!(rr >= 0.0 && rr < (double)nRows && cc >= 0.0 && cc < (double)nCols)) return;
    const int t = (int)rr * nCols + (int)cc;
    const float4 G = J.tg[t];
    const float2 T = J.trg[t];
    A.h[28] += 1.f;
    // saliency: a failed photo OR depth test skips the whole pixel (`continue`, :5319-5320, :5348-5349)
    if (photo && fabsf(G.x) < C.thr_int && fabsf(G.y) < C.thr_int) return;
    if (depth && fabsf(G.z) < C.thr_depth && fabsf(G.w) < C.thr_depth) return;
    // jacobianT36 = Rt^-1(3x3) * [I | -skew(point3D_robot2)] (:5289-5292); the zero products of the
    // 3-term sums drop out exactly
    const float* Ri = J.Rti;   // col-major: Ri(i, j) = Ri[j*4 + i]
    float T36[3][6];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        T36[a][0] = Ri[a]; T36[a][1] = Ri[4 + a]; T36[a][2] = Ri[8 + a];
        T36[a][3] = Ri[4 + a] * (-p2.z) + Ri[8 + a] * p2.y;
        T36[a][4] = Ri[a] * p2.z + Ri[8 + a] * (-p2.x);
        T36[a][5] = Ri[a] * (-p2.y) + Ri[4 + a] * p2.x;
    }
    // jacobianProj23 (:5294-5303), float entries from double expressions
    const float P00 = (float)(J.fxd * inv), P11 = (float)(J.fyd * inv);
    const float P02 = (float)(((-J.fxd * (double)p3.x) * inv) * inv);
    const float P12 = (float)(((-J.fyd * (double)p3.y) * inv) * inv);
    float Jw0[6], Jw1[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        Jw0[k] = P00 * T36[0][k] + P02 * T36[2][k];
        Jw1[k] = P11 * T36[1][k] + P12 * T36[2][k];
    }
    if (photo) {
        const float photoDiff = T.x - gray1;
        const double w = (double)huberf(photoDiff, C.sd_photo) * C.sd_photo_inv_d;
        const float wf = (float)w;
        const float wgx = wf * G.x, wgy = wf * G.y;          // (weight_photo * grad) * jacobianWarpRt
        float Jp[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) Jp[k] = wgx * Jw0[k] + wgy * Jw1[k];
        acc_fma(A, Jp, (float)(w * (double)photoDiff));
    }
    if (depth && isfinite(T.y)) {
        const float depthDiff = T.y - z;
        const float sd = C.sd_depth * z;
        const float w = huberf(depthDiff, sd) / sd;
        float Jd[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) Jd[k] = w * (G.z * Jw0[k] + G.w * Jw1[k]);
        acc_fma(A, Jd, w * depthDiff);
    }
}

template <int METHOD>
__global__ __launch_bounds__(TPB) void k_robot_pass(const RobotJob* __restrict__ jobs, RobotGrid grid, IcpConst C,
                                                    double* __restrict__ partials_all, double* __restrict__ sums,
                                                    unsigned* __restrict__ tickets) {
    __shared__ float s_red[NW][32];
    __shared__ double s_err[NW], s_errd[NW];
    __shared__ double s_fin[RG][32];
    __shared__ int s_last;

    int j = 0;
    while (j + 1 < grid.njobs && (int)blockIdx.x >= grid.block0[j + 1]) ++j;
    const RobotJob& J = jobs[j];
    const int b = (int)blockIdx.x - grid.block0[j];
    const int nb = grid.block0[j + 1] - grid.block0[j];
    double* partials = partials_all + (long)j * R360_ROBOT_MAX_BLOCKS * 32;

    Acc A;
#pragma unroll
    for (int k = 0; k < 32; ++k) A.h[k] = 0.f;
    A.err2 = 0.0;
    A.err2d = 0.0;
    const int npx = J.rows * J.cols;
    for (int i = b * TPB + threadIdx.x; i < npx; i += nb * TPB) {
        const int r = i / J.cols;
        robot_pixel<METHOD>(A, J, C, i, r, i - r * J.cols);
    }

    // wave butterfly -> per-workgroup fp64 record (as k_pin_pass)
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const float mine = wave_reduce_scatter32(A.h, lane);
    const double e2 = wave_sum_d(A.err2);
    const double e2d = wave_sum_d(A.err2d);
    if ((lane & 1) == 0) s_red[wid][scatter_slot(lane)] = mine;
    if (lane == 0) { s_err[wid] = e2; s_errd[wid] = e2d; }
    __syncthreads();
    if (threadIdx.x < 32) {
        double v = 0.0;
        if (threadIdx.x == R360_SUM_ERR2) { for (int w = 0; w < NW; ++w) v += s_err[w]; }
        else if (threadIdx.x == R360_SUM_ERR2D) { for (int w = 0; w < NW; ++w) v += s_errd[w]; }
        else { for (int w = 0; w < NW; ++w) v += (double)s_red[w][threadIdx.x]; }
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(partials) + (long)b * 32 + threadIdx.x,
                           (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(&tickets[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (prev == (unsigned)nb - 1);
    }
    __syncthreads();
    if (!s_last) return;
    {
        const int q = threadIdx.x & 15, g = threadIdx.x >> 4;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(partials, 0, nb * 256, 0x00020000);
        double a0 = 0.0, a1 = 0.0;
        for (int r = g; r < nb; r += RG) {
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, (r * 16 + q) * 16, 0, 16);
            a0 += __longlong_as_double((long long)(((unsigned long long)x[1] << 32) | x[0]));
            a1 += __longlong_as_double((long long)(((unsigned long long)x[3] << 32) | x[2]));
        }
        s_fin[g][2 * q] = a0;
        s_fin[g][2 * q + 1] = a1;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        double t = 0.0;
        for (int g = 0; g < RG; ++g) t += s_fin[g][threadIdx.x];
        sums[j * 32 + threadIdx.x] = t;
        if (threadIdx.x == 0) tickets[j] = 0;
    }
}

// RegisterDensePhotoICP's level loop (RegisterRGBD360.h:387-505) over the pass sums, one wave.
// Job (level l, sensor k) = l * 8 + k.
__global__ __launch_bounds__(64) void k_robot_finalize(const double* __restrict__ sums, int nL,
                                                       RobotOut* __restrict__ out) {
    __shared__ float sH[36], sg[6];
    __shared__ int s_ran;
    const int lane = threadIdx.x;
    if (lane == 0) { out->ok = 1; out->illposed_level = -1; out->any = 0; }
    for (int l = nL - 1; l >= 0; --l) {
        if (lane == 0) {
            // error += calcPhotoICPError_robot(...) over sensors 0..7 (:398-402)
            double error = 0.0;
            for (int k = 0; k < 8; ++k) {
                const double* s = sums + (l * 8 + k) * 32;
                error += s[R360_SUM_ERR2] + s[R360_SUM_ERR2D];
            }
            out->error[l] = error;
            int nvis = 0, nerr = 0;
            for (int k = 0; k < 8; ++k) {
                nvis += (int)sums[(l * 8 + k) * 32 + R360_SUM_NVIS];
                nerr += (int)sums[(l * 8 + k) * 32 + R360_SUM_NVALID];
            }
            out->n_visible[l] = nvis;
            out->n_error[l] = nerr;
            // while(it < maxIters && update_pose.norm() > tol_update && diff_error > tol_residual), with
            // update_pose = (1,...,1) and diff_error = error on entry (:383-388, :410)
            s_ran = error > 0.1;
            out->ran[l] = s_ran;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        if (!s_ran) continue;
        // Hessian += alignSensorID[k].getHessian(), float, sensors in order (:419-424)
        if (lane < 36) {
            const int u = lane / 6, v = lane - (lane / 6) * 6;
            const int a = u < v ? u : v, b = u < v ? v : u;
            const int slot = a * 6 - a * (a - 1) / 2 + (b - a);
            float h = 0.f;
            for (int k = 0; k < 8; ++k) h += (float)sums[(l * 8 + k) * 32 + slot];
            sH[lane] = h;
        }
        if (lane < 6) {
            float gg = 0.f;
            for (int k = 0; k < 8; ++k) gg += (float)sums[(l * 8 + k) * 32 + 21 + lane];
            sg[lane] = gg;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        // (Hessian + lambda * diag(Hessian)).rank() != 6 -> ILL-POSED, return false (:427-434);
        // lambda = 0.001 enters as a float scalar
        float hl = 0.f;
        if (lane < 36) {
            const float h = sH[lane];
            hl = (lane % 7 == 0) ? h + 0.001f * h : h;
        }
        const int rk = wave_rank6(hl, lane);
        if (rk != 6) {
            if (lane == 0) { out->ok = 0; out->illposed_level = l; }
            return;
        }
        // the update and pose_estim_temp (:437-440) are computed and never used: the "new" error is
        // evaluated at pose_estim again, equals `error`, and the loop exits (see the file header)
        if (lane < 36) out->info[lane] = sH[lane];
        if (lane < 6) out->grad[lane] = sg[lane];
        if (lane == 0) out->any = 1;
    }
}

}  // namespace

int launch_robot(r360_ctx* ctx, const RobotJob* d_jobs, const RobotGrid& grid, int method, const IcpConst& C,
                 int finalize_levels) {
    const int slot = timing_begin(ctx, "k_robot_pass");
    const dim3 g(grid.block0[grid.njobs]);
    if (method == R360_PHOTO_CONSISTENCY)
        hipLaunchKernelGGL(k_robot_pass<R360_PHOTO_CONSISTENCY>, g, dim3(TPB), 0, ctx->stream, d_jobs, grid, C,
                           ctx->d_rob_partials, ctx->d_rob_sums, ctx->d_rob_tickets);
    else if (method == R360_DEPTH_CONSISTENCY)
        hipLaunchKernelGGL(k_robot_pass<R360_DEPTH_CONSISTENCY>, g, dim3(TPB), 0, ctx->stream, d_jobs, grid, C,
                           ctx->d_rob_partials, ctx->d_rob_sums, ctx->d_rob_tickets);
    else
        hipLaunchKernelGGL(k_robot_pass<R360_PHOTO_DEPTH>, g, dim3(TPB), 0, ctx->stream, d_jobs, grid, C,
                           ctx->d_rob_partials, ctx->d_rob_sums, ctx->d_rob_tickets);
    timing_end(ctx, slot);
    if (finalize_levels > 0)
        hipLaunchKernelGGL(k_robot_finalize, dim3(1), dim3(64), 0, ctx->stream, ctx->d_rob_sums, finalize_levels,
                           ctx->d_rob_out);
    R360_HIP(hipGetLastError());
    return 0;
}
