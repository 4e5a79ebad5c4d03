// icp_kernels.hip — the fused spherical photometric+geometric ICP pass for gfx950.
//
// One launch = one "pass" of RegisterPhotoICP::alignFrames360 at one pyramid level:
//   errorPhotoICP_sphere (RegisterPhotoICP.h:2545-2739) and calcHessGrad_sphere (:2745-3228)
//   evaluated together at the same pose (they share the transform/projection/gathers), the
//   6x6 JtJ / 6x1 Jtr / error / count sums reduced in two stages (wave butterfly in registers
//   -> LDS across waves -> one fp64 record per workgroup -> the last-arriving workgroup sums the
//   records in a fixed order), and the Gauss-Newton step (:4611-4722) executed by that last
//   workgroup on the device.  No host round trip per iteration: the host enqueues
//   1 + maxIters passes per level and passes after convergence exit at entry.
//
// Memory: per source pixel 8 B ({gray, depth} float2, streamed); per visible pixel 16 B target
// gradients {gx, gy, dgx, dgy} + 8 B target {gray, depth} gathered — the 8N + 24V algorithmic
// bytes of SURVEY.md §8(d).  No Jacobian rows are materialised (the reference writes and
// re-reads imgSize x 6 buffers, :2761-2767).
#include "../r360_internal.h"
#include "../libm_f32.h"

namespace {

constexpr int TPB = 256;
constexpr int NW = TPB / 64;

struct Pose12 { float R[9]; float t[3]; };

__device__ __forceinline__ float huberf(float e, float reg) {  // weightHuber<float> (:545-554)
    const float a = fabsf(e);
    if (a < reg) return 1.f;
    return sqrtf(2 * reg * a - reg * reg) / a;
}

// Accumulator slots: 0..20 upper-triangle H (row-major), 21..26 g, 27 n_valid, 28 n_visible.
struct Acc {
    float h[32];
    double err2;
};

__device__ __forceinline__ void acc_row(Acc& A, const float J[6], float r) {
    A.h[0] += J[0] * J[0];
    A.h[1] += J[0] * J[1];
    A.h[2] += J[0] * J[2];
    A.h[3] += J[0] * J[3];
    A.h[4] += J[0] * J[4];
    A.h[5] += J[0] * J[5];
    A.h[6] += J[1] * J[1];
    A.h[7] += J[1] * J[2];
    A.h[8] += J[1] * J[3];
    A.h[9] += J[1] * J[4];
    A.h[10] += J[1] * J[5];
    A.h[11] += J[2] * J[2];
    A.h[12] += J[2] * J[3];
    A.h[13] += J[2] * J[4];
    A.h[14] += J[2] * J[5];
    A.h[15] += J[3] * J[3];
    A.h[16] += J[3] * J[4];
    A.h[17] += J[3] * J[5];
    A.h[18] += J[4] * J[4];
    A.h[19] += J[4] * J[5];
    A.h[20] += J[5] * J[5];
    A.h[21] += J[0] * r;
    A.h[22] += J[1] * r;
    A.h[23] += J[2] * r;
    A.h[24] += J[3] * r;
    A.h[25] += J[4] * r;
    A.h[26] += J[5] * r;
}

template <int METHOD>
__device__ __forceinline__ void pixel(Acc& A, const Pose12& P, float d, float gray_s, float sp, float cp, float st,
                                      float ct, const float2* __restrict__ trg, const float4* __restrict__ tg,
                                      int nRows, int nCols, float half_nRows, float angle_res_inv,
                                      const IcpConst& C) {
    if (!(C.min_d < d && d < C.max_d)) return;                     // LUT validity (:4578)
    const float lx = d * sp;                                       // LUT_xyz_sphere (:4580-4582)
    const float ly = -d * cp * st;
    const float lz = -d * cp * ct;
    float X = P.R[0] * lx + P.R[1] * ly + P.R[2] * lz; X = X + P.t[0];
    float Y = P.R[3] * lx + P.R[4] * ly + P.R[5] * lz; Y = Y + P.t[1];
    float Z = P.R[6] * lx + P.R[7] * ly + P.R[8] * lz; Z = Z + P.t[2];
    const float dist = sqrtf(X * X + Y * Y + Z * Z);
    const float dist_inv = 1.f / dist;
    const float phi_trg = r360m::asinf(X * dist_inv);        // glibc-exact (libm_f32.h)
    const float theta_trg = (float)((double)r360m::atan2f(Y, Z) + R360_PI);
    // round() + int conversion + the (:2989) bounds test, done on the float values so NaN and
    // out-of-range projections are rejected exactly as the x86 reference's (int) conversion does.
    const float rf = roundf(half_nRows - phi_trg * angle_res_inv);
    const float cf = roundf(theta_trg * angle_res_inv);
    if (!((rf >= 0.f && rf < (float)nRows) && cf < (float)nCols)) return;
    const int r = (int)rf, c = (int)cf;
    A.h[28] += 1.f;                                                 // numVisiblePixels
    const long t = (long)r * nCols + c;
    const float4 G = tg[t];                                         // {gx, gy, dgx, dgy}
    const bool photo = (METHOD == R360_PHOTO_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    const bool depth = (METHOD == R360_DEPTH_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    if (photo && fabsf(G.x) < C.thr_int && fabsf(G.y) < C.thr_int) return;  // 'continue' (:3038)
    const float2 T = trg[t];                                        // {gray, depth} of target
    // jacobianProj23 * jacobianT36 (:2995-3026), jacobianT36 = [I | -skew(p')]
    const float z_inv = 1.f / Z;
    const float z_inv2 = z_inv * z_inv;
    const float D_atan_theta = 1.f / (1 + Y * Y * z_inv2) * angle_res_inv;
    const float P01 = D_atan_theta * z_inv;
    const float P02 = -Y * z_inv2 * D_atan_theta;
    const float dist_inv2 = dist_inv * dist_inv;
    const float x_dist_inv2 = X * dist_inv2;
    const float D_asin = 1.f / sqrtf(1 - X * x_dist_inv2) * angle_res_inv;
    const float P10 = -D_asin * dist_inv * (1 - X * x_dist_inv2);
    const float P11 = D_asin * (x_dist_inv2 * Y * dist_inv);
    const float P12 = D_asin * (x_dist_inv2 * Z * dist_inv);
    // T36 rows: (1,0,0,0,Z,-Y) (0,1,0,-Z,0,X) (0,0,1,Y,-X,0)
    const float T0[6] = {1, 0, 0, 0, Z, -Y};
    const float T1[6] = {0, 1, 0, -Z, 0, X};
    const float T2[6] = {0, 0, 1, Y, -X, 0};
    float Jw0[6], Jw1[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        Jw0[k] = 0.f * T0[k] + P01 * T1[k] + P02 * T2[k];
        Jw1[k] = P10 * T0[k] + P11 * T1[k] + P12 * T2[k];
    }
    if (photo) {
        const float photoDiff = T.x - gray_s;
        const float wh = huberf(photoDiff, C.sd_photo);
        // errorPhotoICP_sphere: double weight, float residual (:2699-2709)
        const float wEd = (float)((double)wh * C.sd_photo_inv_d * photoDiff);
        A.err2 += (double)(wEd * wEd);
        A.h[27] += 1.f;
        // calcHessGrad_sphere: float weight (:3047-3052)
        const float w = wh * C.sd_photo_inv_f;
        const float res = w * photoDiff;
        const float wgx = w * G.x, wgy = w * G.y;
        float J[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) J[k] = wgx * Jw0[k] + wgy * Jw1[k];
        acc_row(A, J, res);
    }
    if (depth) {
        const float depth2 = T.y;
        if (isfinite(depth2)) {
            if (fabsf(G.z) < C.thr_depth && fabsf(G.w) < C.thr_depth) return;  // (:3072-3073)
            const float depthDiff = depth2 - dist;
            const float sd = C.sd_depth * depth2;
            const float w = huberf(depthDiff, sd) / sd;
            const float wE = (float)((double)w * depthDiff);
            A.err2 += (double)(wE * wE);
            A.h[27] += 1.f;
            const float res = w * depthDiff;
            const float js0 = X * dist_inv, js1 = Y * dist_inv, js2 = Z * dist_inv;
            float J[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const float ga = G.z * Jw0[k] + G.w * Jw1[k];
                const float gb = js0 * T0[k] + js1 * T1[k] + js2 * T2[k];
                J[k] = w * (ga - gb);
            }
            acc_row(A, J, res);
        }
    }
}

// Butterfly reduce-scatter of 32 floats across a 64-lane wave: 32 shuffles instead of 32*6.
// On return lane L holds the wave total of slot idx(L) = (bit5 bit4 bit3 bit2 bit1 of L) in a
// fixed bit order, identical for lanes L and L^1.
template <int M, int HALF>
__device__ __forceinline__ void bfly_step(float (&v)[32], int lane) {
    const bool hi = (lane & M) != 0;
#pragma unroll
    for (int j = 0; j < HALF; ++j) {
        const float keep = hi ? v[j + HALF] : v[j];
        const float send = hi ? v[j] : v[j + HALF];
        v[j] = keep + __shfl_xor(send, M, 64);
    }
}

__device__ __forceinline__ float wave_reduce_scatter32(float (&v)[32], int lane) {
    bfly_step<32, 16>(v, lane);
    bfly_step<16, 8>(v, lane);
    bfly_step<8, 4>(v, lane);
    bfly_step<4, 2>(v, lane);
    bfly_step<2, 1>(v, lane);
    return v[0] + __shfl_xor(v[0], 1, 64);
}

__device__ __forceinline__ int scatter_slot(int lane) {
    // step with mask 32 selects the upper half (+16), mask 16 -> +8, ... mask 2 -> +1
    return ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 +
           ((lane >> 1) & 1);
}

__device__ __forceinline__ double wave_sum_d(double x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
}

// ---------------------------------------------------------------- GN step (thread 0 of last block)
#include "icp_gn.inc"

__device__ __forceinline__ double ld_sc1(const double* p) {  // agent-scope (L1-bypassing) load
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <int METHOD>
__global__ __launch_bounds__(TPB) void k_icp_pass(const float2* __restrict__ src, const float2* __restrict__ trg,
                                                 const float4* __restrict__ tg, const float* __restrict__ sinphi,
                                                 const float* __restrict__ cosphi, const float* __restrict__ sinth,
                                                 const float* __restrict__ costh, int nRows, int nCols,
                                                 IcpConst C, IcpState* S, double* __restrict__ partials, int first,
                                                 int eval_only) {
    __shared__ float s_red[NW][32];
    __shared__ double s_err[NW];
    __shared__ double s_fin[8][32];
    __shared__ int s_last;
    __shared__ GnShared s_gn;
    __shared__ IcpState s_state;

    if (S->stop) return;
    if (!first && !S->active && !eval_only) return;

    const float* pm = (first && !eval_only) ? S->pose : S->cand;
    Pose12 P;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) P.R[r * 3 + c] = pm[c * 4 + r];
        P.t[r] = pm[12 + r];
    }
    const float angle_res = (float)(2 * R360_PI / nCols);
    const float angle_res_inv = 1 / angle_res;
    const float half_nRows = (float)(0.5 * nRows - 0.5);

    Acc A;
#pragma unroll
    for (int k = 0; k < 32; ++k) A.h[k] = 0.f;
    A.err2 = 0.0;

    const int units = (nRows * nCols) >> 2;  // 4 pixels of one row per unit (nCols % 4 == 0)
    const float4* src4 = reinterpret_cast<const float4*>(src);
    const float4* st4 = reinterpret_cast<const float4*>(sinth);
    const float4* ct4 = reinterpret_cast<const float4*>(costh);
    const int cq = nCols >> 2;
    for (int u = blockIdx.x * TPB + threadIdx.x; u < units; u += gridDim.x * TPB) {
        const int r = u / cq;
        const int c4 = u - r * cq;
        const float4 a = src4[2 * u], b = src4[2 * u + 1];  // {g0,d0,g1,d1} {g2,d2,g3,d3}
        const float4 s = st4[c4], c = ct4[c4];
        const float sp = sinphi[r], cp = cosphi[r];
        pixel<METHOD>(A, P, a.y, a.x, sp, cp, s.x, c.x, trg, tg, nRows, nCols, half_nRows, angle_res_inv, C);
        pixel<METHOD>(A, P, a.w, a.z, sp, cp, s.y, c.y, trg, tg, nRows, nCols, half_nRows, angle_res_inv, C);
        pixel<METHOD>(A, P, b.y, b.x, sp, cp, s.z, c.z, trg, tg, nRows, nCols, half_nRows, angle_res_inv, C);
        pixel<METHOD>(A, P, b.w, b.z, sp, cp, s.w, c.w, trg, tg, nRows, nCols, half_nRows, angle_res_inv, C);
    }

    // ---- stage 1: wave butterfly (f32) -> LDS -> per-workgroup fp64 record
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const float mine = wave_reduce_scatter32(A.h, lane);
    const double e2 = wave_sum_d(A.err2);
    if ((lane & 1) == 0) s_red[wid][scatter_slot(lane)] = mine;
    if (lane == 0) s_err[wid] = e2;
    __syncthreads();
    if (threadIdx.x < 32) {
        double v;
        if (threadIdx.x == R360_SUM_ERR2) {
            v = 0; for (int w = 0; w < NW; ++w) v += s_err[w];
        } else {
            v = 0; for (int w = 0; w < NW; ++w) v += (double)s_red[w][threadIdx.x];
        }
        // write-through (sc1) store: visible at agent scope without an L2 write-back fence
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(partials) + (long)blockIdx.x * 32 + threadIdx.x,
                           (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // ---- stage 2: arrival ticket; the last workgroup reduces all records and runs the GN step
    // Hand-off (MI355X_MICROARCH.md 'Valid forms', row 1): every record store is sc1 and drained by
    // its wave (vmcnt(0) above) before the barrier; one relaxed agent-scope add per workgroup; the
    // last adder reads every record with sc1 loads.  No buffer_wbl2 / buffer_inv fences: a release
    // fence per workgroup wrote back each XCD's dirty L2 (tens of us per pass).
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(&S->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (prev == gridDim.x - 1);
    }
    __syncthreads();
    if (!s_last) return;
    {
        // fixed-order reduction of the per-workgroup records; 8 independent accumulators per thread
        // keep 8 loads in flight (the serial chain of dependent loads was the finalize's cost)
        const int v = threadIdx.x & 31, grp = threadIdx.x >> 5;  // 8 groups of 32
        double a8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int nb = (int)gridDim.x;
        int bk = grp;
        for (; bk + 56 < nb; bk += 64) {
#pragma unroll
            for (int j = 0; j < 8; ++j) a8[j] += ld_sc1(partials + (long)(bk + 8 * j) * 32 + v);
        }
        for (int j = 0; bk < nb; bk += 8, ++j) a8[j & 7] += ld_sc1(partials + (long)bk * 32 + v);
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += a8[j];
        s_fin[grp][v] = acc;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        double t = 0.0;
        for (int g = 0; g < 8; ++g) t += s_fin[g][threadIdx.x];
        s_fin[0][threadIdx.x] = t;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        if (eval_only) {
            if (threadIdx.x < 32) S->sums[threadIdx.x] = s_fin[0][threadIdx.x];
        } else {
            // Stage the whole state in LDS with one coalesced 16-B access per lane, run the step on
            // the LDS copy (a single lane walking global memory serialises ~150 dependent accesses,
            // ~35 us), then write it back the same way.
            constexpr int NQ = (int)(sizeof(IcpState) / 16);
            uint4* sq = reinterpret_cast<uint4*>(&s_state);
            const uint4* gq = reinterpret_cast<const uint4*>(S);
            for (int q = threadIdx.x; q < NQ; q += 64) sq[q] = gq[q];
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            gn_step_wave(&s_state, s_fin[0], C, first, &s_gn, threadIdx.x);
            if (threadIdx.x == 0) s_state.ticket = 0;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            uint4* wq = reinterpret_cast<uint4*>(S);
            for (int q = threadIdx.x; q < NQ; q += 64) wq[q] = sq[q];
        }
        if (eval_only && threadIdx.x == 0) S->ticket = 0;
    }
}

}  // namespace

namespace {
__global__ void k_libm(const float* x, const float* y, const float* z, int n, float* as, float* at) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { as[i] = r360m::asinf(x[i]); at[i] = r360m::atan2f(y[i], z[i]); }
}
}  // namespace

// Test hook: evaluates the asinf/atan2f port on the host or on the device.
extern "C" int r360_libm_eval(const float* x, const float* y, const float* z, int n, float* asin_out,
                              float* atan2_out, int on_device) {
    if (!on_device) {
        for (int i = 0; i < n; ++i) { asin_out[i] = r360m::asinf(x[i]); atan2_out[i] = r360m::atan2f(y[i], z[i]); }
        return 0;
    }
    float* d = nullptr;
    const size_t b = sizeof(float) * (size_t)n;
    R360_HIP(hipMalloc(&d, 5 * b));
    R360_HIP(hipMemcpy(d, x, b, hipMemcpyHostToDevice));
    R360_HIP(hipMemcpy(d + n, y, b, hipMemcpyHostToDevice));
    R360_HIP(hipMemcpy(d + 2 * (size_t)n, z, b, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_libm, dim3((n + 255) / 256), dim3(256), 0, 0, d, d + n, d + 2 * (size_t)n, n,
                       d + 3 * (size_t)n, d + 4 * (size_t)n);
    R360_HIP(hipGetLastError());
    R360_HIP(hipMemcpy(asin_out, d + 3 * (size_t)n, b, hipMemcpyDeviceToHost));
    R360_HIP(hipMemcpy(atan2_out, d + 4 * (size_t)n, b, hipMemcpyDeviceToHost));
    R360_HIP(hipFree(d));
    return 0;
}

int icp_blocks_for(int n_pixels) {
    const int units = n_pixels / 4;
    int b = (units + TPB * 2 - 1) / (TPB * 2);
    if (b > 1024) b = 1024;
    return b < 1 ? 1 : b;
}

int launch_icp_level(r360_ctx* ctx, const r360_frame* trg, const r360_frame* src, int level, int method,
                     const IcpConst& C, int first, int eval_only) {
    const LevelBufs& Ls = src->lv[level];
    const LevelBufs& Lt = trg->lv[level];
    const LevelTrig& T = src->calib->trig[level];
    const int nb = icp_blocks_for(Ls.rows * Ls.cols);
    const char* name = level == 0 ? "k_icp_pass_L0" : "k_icp_pass";
    const int slot = timing_begin(ctx, name);
#define R360_LAUNCH(M)                                                                                       \
    hipLaunchKernelGGL(k_icp_pass<M>, dim3(nb), dim3(TPB), 0, ctx->stream, Ls.p0, Lt.p0, Lt.tg, T.sinphi,   \
                       T.cosphi, T.sinth, T.costh, Ls.rows, Ls.cols, C, ctx->d_state, ctx->d_partials, first, \
                       eval_only)
    if (method == R360_PHOTO_CONSISTENCY) R360_LAUNCH(R360_PHOTO_CONSISTENCY);
    else if (method == R360_DEPTH_CONSISTENCY) R360_LAUNCH(R360_DEPTH_CONSISTENCY);
    else R360_LAUNCH(R360_PHOTO_DEPTH);
#undef R360_LAUNCH
    timing_end(ctx, slot);
    R360_HIP(hipGetLastError());
    return 0;
}
