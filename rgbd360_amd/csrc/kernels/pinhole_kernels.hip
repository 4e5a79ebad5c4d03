// pinhole_kernels.hip — §8(f) rank 3: RegisterPhotoICP's per-sensor pinhole dense registration on gfx950.
//
//   errorPhotoICP   include/RegisterPhotoICP.h:560-761  (LUT branch; LUT of alignFrames :4285-4298)
//   calcHessGrad    :767-1100
//   alignFrames     :4254-4512  (Levenberg-Marquardt: lambda 0.01, step 10, one LM retry)
//
// One fused pass per candidate pose evaluates errorPhotoICP AND calcHessGrad (the H / g of an accepted
// candidate are the next iteration's), exactly like the spherical pass of icp_kernels.hip.  Up to 8
// independent alignments (one per sensor: the Methods harness's single-sensor mode on every sensor of
// a Frame360 pair, MethodsRegisterRGBD360.cpp:320-345) run in the same launch, blockIdx.y = job, each
// with its own device state, record area and arrival ticket; the last workgroup of a job runs the
// LM step for that job.  Small per-sensor images (QVGA: 76800 px) would leave most of the 256 CUs idle
// one at a time; eight at once fill the chip.
//
// Exactness: the LUT, transform, 1/z, projection and rounding are the reference's float expressions
// (-ffp-contract=off), so visibility, target pixels, counts and the error terms are exact; H / g are
// float-accumulated like the reference's (omp critical, :1080-1097) and compared within tolerance.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>

#include "../r360_internal.h"

namespace {

constexpr int TPB = 256;
constexpr int NW = TPB / 64;
constexpr int RG = TPB / 16;   // record-reduction groups (16 lanes x 16 B per record)

#include "icp_common.inc"
#include "icp_la.inc"

struct Pose12 { float R[9]; float t[3]; };

// alignFrames' own LM constants (:4301-4312)
constexpr double kLambda0 = 0.01, kStep = 10, kTolResidual = 1e-4, kTolUpdate = 1e-4;
constexpr int kMaxIters = 10;

struct Intr { float fx, fy, ox, oy, inv_fx, inv_fy; };

struct PinProj { float X, Y, Z, inv, gray_s; int t; bool vis; };

// LUT (:4287-4298), rotation * LUT + translation and the projection (:700-714)
__device__ __forceinline__ PinProj pin_project(const Pose12& P, float z, float gray_s, int r, int c, const Intr& I,
                                               int nRows, int nCols, const IcpConst& C) {
    PinProj o;
    const bool valid = (C.min_d < z && z < C.max_d);
    const float lx = ((float)c - I.ox) * z * I.inv_fx;
    const float ly = ((float)r - I.oy) * z * I.inv_fy;
    float X = P.R[0] * lx + P.R[1] * ly + P.R[2] * z; X = X + P.t[0];
    float Y = P.R[3] * lx + P.R[4] * ly + P.R[5] * z; Y = Y + P.t[1];
    float Z = P.R[6] * lx + P.R[7] * ly + P.R[8] * z; Z = Z + P.t[2];
    const float inv = 1.f / Z;                               // (float)(1.0/Z): the same rounding
    const float tc = (X * I.fx) * inv + I.ox;
    const float tr = (Y * I.fy) * inv + I.oy;
    const float rf = roundf(tr), cf = roundf(tc);
    // (int)round(.) and the bounds test; the float comparisons reject NaN / huge values exactly as the
    // x86 conversion (INT_MIN) does
    o.vis = valid && rf >= 0.f && rf < (float)nRows && cf >= 0.f && cf < (float)nCols;
    o.t = o.vis ? (int)rf * nCols + (int)cf : 0;
    o.X = X; o.Y = Y; o.Z = Z; o.inv = inv; o.gray_s = gray_s;
    return o;
}

// Error terms (errorPhotoICP) and Jacobian rows (calcHessGrad) of one source pixel, branch-free:
// skipped terms go through selects, never a multiply by 0.
//   slots: 0..26 H / g, 27 nValidPhotoPts, 28 visible, 29 nValidDepthPts; err2 = PhotoResidual,
//   err2d = DepthResidual
template <int METHOD>
__device__ __forceinline__ void pin_contribute(Acc& A, const PinProj& o, const float4 G, const float2 T, const Intr& I,
                                               const IcpConst& C) {
    constexpr bool photo = (METHOD == R360_PHOTO_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    constexpr bool depth = (METHOD == R360_DEPTH_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    const float X = o.X, Y = o.Y, Z = o.Z, inv = o.inv;
    const bool vis = o.vis;
    const bool fin_d = isfinite(T.y);
    // errorPhotoICP (:716-752): no saliency test
    const float photoDiff = T.x - o.gray_s;
    const float wp = huberf(photoDiff, C.sd_photo) * C.sd_photo_inv_f;
    const float wEp = wp * photoDiff;
    const float depthDiff = T.y - Z;
    const float sd = C.sd_depth * Z;
    const float wd = huberf(depthDiff, sd) / sd;
    const float wEd = wd * depthDiff;
    A.h[28] += vis ? 1.f : 0.f;
    if (photo) { A.err2 += vis ? (double)(wEp * wEp) : 0.0; A.h[27] += vis ? 1.f : 0.f; }
    if (depth) { A.err2d += (vis && fin_d) ? (double)(wEd * wEd) : 0.0; A.h[29] += (vis && fin_d) ? 1.f : 0.f; }
    // calcHessGrad: a failed photo OR depth saliency test skips the whole point (:1031-1032, :1056-1057)
    const bool sal_p = !(fabsf(G.x) < C.thr_int && fabsf(G.y) < C.thr_int);
    const bool sal_d = !(fabsf(G.z) < C.thr_depth && fabsf(G.w) < C.thr_depth);
    const bool keep = vis && (!photo || sal_p) && (!depth || sal_d);
    float Jw0[6], Jw1[6];
    {
#pragma clang fp contract(fast)
        // jacobianWarpRt (:993-1010)
        const float inv2 = inv * inv;
        Jw0[0] = I.fx * inv;        Jw1[0] = 0.f;
        Jw0[1] = 0.f;               Jw1[1] = I.fy * inv;
        Jw0[2] = -I.fx * X * inv2;  Jw1[2] = -I.fy * Y * inv2;
        Jw0[3] = -I.fx * Y * X * inv2;
        Jw1[3] = -I.fy * (1 + Y * Y * inv2);
        Jw0[4] = I.fx * (1 + X * X * inv2);
        Jw1[4] = I.fy * X * Y * inv2;
        Jw0[5] = -I.fx * Y * inv;   Jw1[5] = I.fy * X * inv;
    }
    if (photo) {
#pragma clang fp contract(fast)
        const bool jp = keep;
        const float wgx = wp * G.x, wgy = wp * G.y;                         // (w * grad) * Jw (:1045)
        float J[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) J[k] = jp ? wgx * Jw0[k] + wgy * Jw1[k] : 0.f;
        acc_fma(A, J, jp ? wEp : 0.f);
    }
    if (depth) {
#pragma clang fp contract(fast)
        const bool jd = keep && fin_d;
        // w * (dgrad * Jw - jacobianRt_z), jacobianRt_z = (0, 0, 1, Y, -X, 0) (:1072-1073)
        float J[6];
        J[0] = G.z * Jw0[0] + G.w * Jw1[0];
        J[1] = G.z * Jw0[1] + G.w * Jw1[1];
        J[2] = G.z * Jw0[2] + G.w * Jw1[2] - 1.f;
        J[3] = G.z * Jw0[3] + G.w * Jw1[3] - Y;
        J[4] = G.z * Jw0[4] + G.w * Jw1[4] + X;
        J[5] = G.z * Jw0[5] + G.w * Jw1[5];
#pragma unroll
        for (int k = 0; k < 6; ++k) J[k] = jd ? wd * J[k] : 0.f;
        acc_fma(A, J, jd ? wEd : 0.f);
    }
}

struct LmShared {
    double x[6]; double A[42];
    float Hc[36]; float gc[6]; float Hs[36]; float gs[6]; float P[16];
    float lam;      // damping of the pending solve (0: undamped step + rank test)
    int mode;       // 0 stop, 1 rank test + undamped step (:4345-4358), 2 damped LM retry (:4388-4391)
};

// One alignFrames loop transition after a pass (wave 0 of the job's last workgroup; lane 0 writes the
// state).  The pass evaluated errorPhotoICP + calcHessGrad at S->pose (first pass of a level) or at the
// pending candidate S->cand.
__device__ void lm_step_wave(IcpState* S, const double* sums, const IcpConst& C, int first, LmShared* G, int lane) {
    const double nD = sums[R360_SUM_NDEPTH];
    // avPhotoResidual = sqrt(PhotoResidual / nValidDepthPts) (:760), + avDepthResidual (:761-762)
    const double new_err = sqrt(sums[R360_SUM_ERR2] / nD) + sqrt(sums[R360_SUM_ERR2D] / nD);
    if (lane < 36) {
        const int u = lane / 6, v = lane - (lane / 6) * 6;
        const int a = u < v ? u : v, b = u < v ? v : u;
        G->Hc[lane] = (float)sums[a * 6 - a * (a - 1) / 2 + (b - a)];
    }
    if (lane < 6) G->gc[lane] = (float)sums[21 + lane];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (lane == 0) {
        S->passes++;
        // errorPhotoICP assigns the residual members (:759-762); avResidual is float
        S->av_photo = sqrt(sums[R360_SUM_ERR2] / nD);
        S->av_depth = sqrt(sums[R360_SUM_ERR2D] / nD);
        S->av_res = (float)(S->av_photo + S->av_depth);
        S->av_set |= 3;
        bool check = false;
        int mode = 0;
        auto accept = [&]() {
            for (int k = 0; k < 16; ++k) S->pose[k] = S->cand[k];
            S->error = new_err;
            S->it = S->it + 1;
            for (int k = 0; k < 36; ++k) S->Hcur[k] = G->Hc[k];
            for (int k = 0; k < 6; ++k) S->gcur[k] = G->gc[k];
        };
        if (first) {                                     // level start: error(pose_estim) (:4316-4321)
            S->error = new_err; S->diff_error = new_err;
            for (int k = 0; k < 6; ++k) S->upd[k] = 1.f;
            S->it = 0; S->loops = 0; S->evals = 0;
            S->lm_lambda = kLambda0; S->lm_phase = 0;
            for (int k = 0; k < 36; ++k) S->Hcur[k] = G->Hc[k];
            for (int k = 0; k < 6; ++k) S->gcur[k] = G->gc[k];
            check = true;
        } else {
            S->evals++;
            const double diff = S->error - new_err;      // :4371, :4400
            S->diff_error = diff;
            if (S->lm_phase == 0) {
                if (diff > 0) {                          // :4374-4380
                    S->lm_lambda = S->lm_lambda / kStep;
                    accept();
                    check = true;
                } else {                                 // :4385-4391: one LM retry from the same pose
                    S->lm_lambda = S->lm_lambda * kStep;
                    mode = 2;
                }
            } else {
                if (diff > 0) accept();                  // :4403-4408
                check = true;                            // LM_maxIters = 1
            }
        }
        if (check) {
            float nu = 0.f;
            for (int k = 0; k < 6; ++k) nu += S->upd[k] * S->upd[k];
            nu = sqrtf(nu);
            const bool cont = S->it < kMaxIters && nu > kTolUpdate && S->diff_error > kTolResidual;   // :4324
            if (!cont) {
                S->active = 0;
                S->iters[C.level] = S->it;
                S->evals_l[C.level] = S->evals;
            } else {
                S->loops++;
                // "Assign the temporal values for the residuals" at the loop iteration's start (:4329-4332)
                S->av_photo_t = S->av_photo; S->av_depth_t = S->av_depth; S->av_res_t = S->av_res;
                S->av_set |= 12;
                for (int k = 0; k < 36; ++k) S->Hout[k] = S->Hcur[k];   // `hessian` of this iteration
                for (int k = 0; k < 6; ++k) S->gout[k] = S->gcur[k];
                mode = 1;
            }
        }
        if (mode) {
            for (int k = 0; k < 36; ++k) G->Hs[k] = S->Hcur[k];
            for (int k = 0; k < 6; ++k) G->gs[k] = S->gcur[k];
            for (int k = 0; k < 16; ++k) G->P[k] = S->pose[k];
        }
        G->lam = (float)S->lm_lambda;                    // Eigen: double * Matrix<float> -> float scalar
        G->mode = mode;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int mode = G->mode;
    if (!mode) return;
    // hessian + lambda * diag(hessian), in float
    auto damped = [&](int i, int j) {
        const float h = G->Hs[i * 6 + j];
        return i == j ? h + G->lam * h : h;
    };
    if (mode == 1) {                                     // (H + lambda diag H).rank() != 6 -> ILL-POSED
        const float hl = lane < 36 ? damped(lane / 6, lane - (lane / 6) * 6) : 0.f;
        if (wave_rank6(hl, lane) != 6) {
            if (lane == 0) {
                S->illposed = 1; S->stop = 1; S->active = 0;
                S->iters[C.level] = S->it;
                S->evals_l[C.level] = S->evals;
            }
            return;
        }
    }
    double aug = 0.0;
    if (lane < 42) {
        const int i = lane / 7, j = lane - (lane / 7) * 7;
        aug = j < 6 ? (double)(mode == 1 ? G->Hs[i * 6 + j] : damped(i, j)) : -(double)G->gs[i];
    }
    wave_solve6(aug, lane, G->x, G->A);
    if (lane == 0) {
        double ud[6];
        for (int k = 0; k < 6; ++k) { S->upd[k] = (float)G->x[k]; ud[k] = S->upd[k]; }
        float E[16];
        exp_se3(ud, 0, E);                               // CPose3D::exp, true SE(3) (:4358, :4391)
        float P[16];
        for (int k = 0; k < 16; ++k) P[k] = G->P[k];
        float Cn[16];
        matmul4f(E, P, Cn);
        for (int k = 0; k < 16; ++k) S->cand[k] = Cn[k];
        S->lm_phase = mode == 2 ? 1 : 0;
        S->active = 1;
    }
}

template <int METHOD>
__global__ __launch_bounds__(TPB) void k_pin_pass(const float2* __restrict__ src_all, const float2* __restrict__ trg_all,
                                                  const float4* __restrict__ tg_all, int nRows, int nCols, IcpConst C,
                                                  Intr I, PinJobs J, IcpState* __restrict__ states,
                                                  double* __restrict__ partials_all, int first, int eval_only) {
    __shared__ float s_red[NW][32];
    __shared__ double s_err[NW], s_errd[NW];
    __shared__ double s_fin[RG][32];
    __shared__ int s_last;
    __shared__ LmShared s_lm;
    __shared__ IcpState s_state;

    const int job = blockIdx.y;
    IcpState* S = states + job;
    if (S->stop) return;
    if (!first && !S->active && !eval_only) return;
    const long img = (long)J.sensor[job] * nRows * nCols;
    const float2* src = src_all + img;
    const float2* trg = trg_all + img;
    const float4* tg = tg_all + img;
    double* partials = partials_all + (long)job * R360_PIN_MAX_BLOCKS * 32;

    const float* pm = (first && !eval_only) ? S->pose : S->cand;
    Pose12 P;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) P.R[r * 3 + c] = pm[c * 4 + r];
        P.t[r] = pm[12 + r];
    }
    Acc A;
#pragma unroll
    for (int k = 0; k < 32; ++k) A.h[k] = 0.f;
    A.err2 = 0.0;
    A.err2d = 0.0;

    const int npx = nRows * nCols;
    const int stride = gridDim.x * TPB;
    // two pixels in flight per thread: project both, issue both gathers, then the math
    int i = blockIdx.x * TPB + threadIdx.x;
    for (; i + stride < npx; i += 2 * stride) {
        const int i1 = i + stride;
        const float2 a0 = src[i], a1 = src[i1];
        const int r0 = i / nCols, r1 = i1 / nCols;
        const PinProj o0 = pin_project(P, a0.y, a0.x, r0, i - r0 * nCols, I, nRows, nCols, C);
        const PinProj o1 = pin_project(P, a1.y, a1.x, r1, i1 - r1 * nCols, I, nRows, nCols, C);
        const float4 G0 = tg[o0.t], G1 = tg[o1.t];
        const float2 T0 = trg[o0.t], T1 = trg[o1.t];
        pin_contribute<METHOD>(A, o0, G0, T0, I, C);
        pin_contribute<METHOD>(A, o1, G1, T1, I, C);
    }
    if (i < npx) {
        const float2 a0 = src[i];
        const int r0 = i / nCols;
        const PinProj o0 = pin_project(P, a0.y, a0.x, r0, i - r0 * nCols, I, nRows, nCols, C);
        pin_contribute<METHOD>(A, o0, tg[o0.t], trg[o0.t], I, C);
    }

    // ---- stage 1: wave butterfly (f32) -> LDS -> per-workgroup fp64 record
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
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(partials) + (long)blockIdx.x * 32 + threadIdx.x,
                           (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // ---- stage 2: arrival ticket of this job; its last workgroup reduces the records (same hand-off as
    // the spherical pass: sc1 record stores drained before the barrier, sc1 loads by the last adder)
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(&S->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (prev == gridDim.x - 1);
    }
    __syncthreads();
    if (!s_last) return;
    {
        const int q = threadIdx.x & 15, g = threadIdx.x >> 4;
        const int nb = (int)gridDim.x;
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
        s_fin[0][threadIdx.x] = t;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        if (eval_only) {
            if (threadIdx.x < 32) S->sums[threadIdx.x] = s_fin[0][threadIdx.x];
            if (threadIdx.x == 0) S->ticket = 0;
        } else {
            constexpr int NQ = (int)(sizeof(IcpState) / 16);
            uint4* sq = reinterpret_cast<uint4*>(&s_state);
            const uint4* gq = reinterpret_cast<const uint4*>(S);
            for (int q = threadIdx.x; q < NQ; q += 64) sq[q] = gq[q];
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            lm_step_wave(&s_state, s_fin[0], C, first, &s_lm, threadIdx.x);
            if (threadIdx.x == 0) s_state.ticket = 0;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            uint4* wq = reinterpret_cast<uint4*>(S);
            for (int q = threadIdx.x; q < NQ; q += 64) wq[q] = sq[q];
        }
    }
}


}  // namespace

// One pass of the batched pinhole alignment at `level` (jobs = J.n sensors).
int launch_pin_level(r360_ctx* ctx, const r360_frame* trg, const r360_frame* src, int level, int method,
                     const IcpConst& C, const float K[4], const PinJobs& J, int first, int eval_only) {
    const LevelBufs& Ls = src->sp[level];
    const LevelBufs& Lt = trg->sp[level];
    // scaleFactor = 1.0/pow(2, level); fx = cameraMatrix(0,0)*scaleFactor ... (:4273-4279)
    const float sc = (float)(1.0 / pow(2, level));
    Intr I;
    I.fx = K[0] * sc; I.fy = K[1] * sc; I.ox = K[2] * sc; I.oy = K[3] * sc;
    I.inv_fx = (float)(1. / I.fx); I.inv_fy = (float)(1. / I.fy);
    static const int ppt = R360_KNOB("R360_PIN_PPT", 4);   // pixels per thread
    const int npx = Ls.rows * Ls.cols;
    int nb = (npx + TPB * ppt - 1) / (TPB * ppt);
    if (nb < 1) nb = 1;
    if (nb > R360_PIN_MAX_BLOCKS) nb = R360_PIN_MAX_BLOCKS;
    const dim3 grid(nb, J.n);
    const int slot = timing_begin(ctx, level == 0 ? "k_pin_pass_L0" : "k_pin_pass");
    if (method == R360_PHOTO_CONSISTENCY)
        hipLaunchKernelGGL(k_pin_pass<R360_PHOTO_CONSISTENCY>, grid, dim3(TPB), 0, ctx->stream, Ls.p0, Lt.p0, Lt.tg,
                           Ls.rows, Ls.cols, C, I, J, ctx->d_pin_state, ctx->d_pin_partials, first, eval_only);
    else if (method == R360_DEPTH_CONSISTENCY)
        hipLaunchKernelGGL(k_pin_pass<R360_DEPTH_CONSISTENCY>, grid, dim3(TPB), 0, ctx->stream, Ls.p0, Lt.p0, Lt.tg,
                           Ls.rows, Ls.cols, C, I, J, ctx->d_pin_state, ctx->d_pin_partials, first, eval_only);
    else
        hipLaunchKernelGGL(k_pin_pass<R360_PHOTO_DEPTH>, grid, dim3(TPB), 0, ctx->stream, Ls.p0, Lt.p0, Lt.tg,
                           Ls.rows, Ls.cols, C, I, J, ctx->d_pin_state, ctx->d_pin_partials, first, eval_only);
    timing_end(ctx, slot);
    R360_HIP(hipGetLastError());
    return 0;
}
