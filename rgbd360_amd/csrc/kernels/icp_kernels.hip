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
#include <cstdio>
#include <type_traits>
#include "../r360_internal.h"
#include "../libm_f32.h"

namespace {

#ifndef R360_ICP_TPB
#define R360_ICP_TPB 256
#endif
#ifndef R360_PK_ACC
#define R360_PK_ACC 0   // PF 6 sums J J^T with packed FMAs (contribute_pk)
#endif
#ifndef R360_ICP_MINB
#define R360_ICP_MINB 5   // waves per SIMD (HIP launch_bounds 2nd arg): caps the pass at 102 VGPRs (94 used)
#endif
// 4 waves per workgroup, 5 workgroups per CU: 5 waves per SIMD (a 512-thread workgroup holds 2 waves per
// SIMD, so 94 VGPRs still gave 4); with 512 workgroups per pass each wave streams twice the chunks, and a
// batched launch (16 pairs) keeps every SIMD at 5 waves (17.8 vs 20.4 us per pair-pass, profiles/r2_v2)
constexpr int TPB = R360_ICP_TPB;
constexpr int NW = TPB / 64;
constexpr int RG = TPB / 16;  // record-reduction groups (16 lanes x 16 B per record)
// the two-level record sum maps ticket group g to the final-stage row g (threadIdx.x >> 4) and sums rows k < RG
static_assert(!R360_GROUP_SUM || R360_TICKET_GROUPS == RG, "R360_GROUP_SUM needs R360_TICKET_GROUPS == TPB / 16");
// gn_step_block (icp_gn.inc) runs the rank test on wave 1 and the solve on wave 2 of the step's workgroup
static_assert(NW >= 3, "the GN step needs at least 3 waves per workgroup (R360_ICP_TPB >= 192)");

struct Pose12 { float R[9]; float t[3]; };

// Target gathers go through buffer loads (32-bit byte offsets, descriptor in SGPRs).  Besides the
// smaller address arithmetic, an intrinsic load is not merged by InstCombine with the loop-carried
// copy of the previous iteration's gather (phi(load a, load b) -> load(phi(a, b)) for plain loads),
// which had moved every gather next to its use and exposed its full latency once per pixel.
struct Gather {
    __amdgpu_buffer_rsrc_t tg, trg;
#ifdef R360_EXP_NOGATHER   // experiment builds only (tools/exp_variants.sh): no target loads
    __device__ __forceinline__ float4 g(int t) const { const float v = (float)(t & 1023) * 1e-3f; return make_float4(v, -v, v, 0.5f * v); }
    __device__ __forceinline__ float2 T(int t) const { return make_float2((float)(t & 255) * 4e-3f, 2.f); }
#else
    __device__ __forceinline__ float4 g(int t) const {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(tg, t * 16, 0, 0);
        return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    }
    __device__ __forceinline__ float2 T(int t) const {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(trg, t * 8, 0, 0);
        return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
    }
#endif
};

#ifdef R360_STAMPS
__device__ unsigned long long g_blk_stamps[3][8192];  // per-workgroup start / loop end / XCC_ID:HW_ID (diagnostic build)
#endif

#include "icp_common.inc"

// occlusion flags per source pixel (k_occ_resolve): bit 0 accepted by the target Z-buffer (a prefix
// maximum of 1/|p'| in LUT order), bit 1 the last accepted point of its target pixel, bit 2 the last
// point (after the Occ2 depth-outlier filter) of its target pixel
enum { OCC_ACC = 1, OCC_OWN = 2, OCC_WIN = 4 };

// ---------------------------------------------------------------- per-pixel pipeline
// Exact part: LUT point, transform and spherical projection, bit-identical to the reference
// (same float expressions, glibc-exact asinf/atan2f, IEEE sqrt/div).  Everything that decides WHICH
// target pixel is read, and the error terms, stays exact; only the Jacobian uses fast rcp/rsq.
struct Proj {
    float X, Y, Z, dist, dist_inv, gray_s;
    int t;          // target pixel index (0 when not visible)
    bool vis;       // valid source depth and projected inside the target image
    bool fix;       // near a rounding boundary: project_fix decides the pixel exactly
};

// Guard bands (pixels) around the .5 rounding boundaries inside which the fast projection defers to the
// exact one.  Worst-case fast-vs-exact differences at level 0 of a 3840-column sphere: row 2e-4 px
// (asin of a ~2-ulp argument, |phi| <= pi/2 rows in view), column 7.5e-4 px (two reciprocal-based
// divisions in atan2 plus the float rounding of theta + pi); coarser levels scale them down.
constexpr float kGuardRow = 6e-4f, kGuardCol = 1.5e-3f;

// What asinf_fast_view returns for |x| >= 0.53 (|phi| >= 32 deg): 1 (a row outside the image) when the
// sphere's half-height nRows * pi / nCols stays below 0.55 rad (the stitched sphere's 30 deg, at every
// pyramid level), NaN otherwise (a taller r360_calib_create_sphere sphere: the lane is deferred to the
// exact projection).
__device__ __forceinline__ float asin_out_for(int nRows, int nCols) {
    return (float)nRows * 3.14159265f < 0.55f * (float)nCols ? 1.0f : __builtin_nanf("");
}

// round() + int conversion + the (:2989) bounds test, on the float values so NaN and out-of-range
// projections are rejected exactly as the x86 reference's (int) conversion does.
__device__ __forceinline__ void set_pixel(Proj& o, float rr, float cc, bool valid, int nRows, int nCols) {
    const float rf = roundf(rr);
    const float cf = roundf(cc);
    o.vis = valid && (rf >= 0.f && rf < (float)nRows) && cf < (float)nCols;
    o.t = o.vis ? (int)rf * nCols + (int)cf : 0;
}

// Branch-free fast projection: the lanes whose coordinates land inside a guard band of a rounding
// boundary (or whose fast path produced NaN, at the poles) are flagged in o.fix and re-projected
// exactly by project_fix before their target pixel is used.  Keeping this part branch-free lets the
// scheduler interleave it with the accumulation of the previous chunk.
template <bool FASTD = false>
__device__ __forceinline__ Proj project(const Pose12& P, float d, float gray_s, float sp, float cp, float st, float ct,
                                        int nRows, int nCols, float half_nRows, float angle_res_inv, const IcpConst& C) {
    Proj o;
    const bool valid = (C.min_d < d && d < C.max_d);                // LUT validity (:4578)
    const float lx = d * sp;                                       // LUT_xyz_sphere (:4580-4582)
    const float ly = -d * cp * st;
    const float lz = -d * cp * ct;
    float X = P.R[0] * lx + P.R[1] * ly + P.R[2] * lz; X = X + P.t[0];
    float Y = P.R[3] * lx + P.R[4] * ly + P.R[5] * lz; Y = Y + P.t[1];
    float Z = P.R[6] * lx + P.R[7] * ly + P.R[8] * lz; Z = Z + P.t[2];
    const float d2 = X * X + Y * Y + Z * Z;
    // |p'| is exact (it enters the depth residual); the projection itself uses hardware rsq/rcp
    const float dist = FASTD ? __builtin_amdgcn_sqrtf(d2) : sqrtf(d2);
    const float dist_inv = __builtin_amdgcn_rsqf(d2);
    const float phi_trg = r360m::asinf_fast(X * dist_inv);
    const float theta_trg = (float)((double)r360m::atan2f_fast(Y, Z) + R360_PI);
    const float rr = half_nRows - phi_trg * angle_res_inv;
    const float cc = theta_trg * angle_res_inv;
    const float gr = fabsf(rr - floorf(rr) - 0.5f), gc = fabsf(cc - floorf(cc) - 0.5f);
    o.fix = valid && !(gr >= kGuardRow && gc >= kGuardCol);          // also catches a NaN of the fast path
    set_pixel(o, rr, cc, valid, nRows, nCols);
    o.X = X; o.Y = Y; o.Z = Z; o.dist = dist; o.dist_inv = dist_inv; o.gray_s = gray_s;
    return o;
}

// Exact re-projection of the flagged lanes: the reference's float expressions with glibc-exact
// asinf/atan2f and IEEE sqrt/div decide the pixel.  Returns whether any lane of the wave changed
// its target pixel (the caller then re-issues the gathers).
__device__ __forceinline__ bool project_fix(Proj& o, int nRows, int nCols, float half_nRows, float angle_res_inv) {
    if (!__any(o.fix)) return false;
    bool changed = false;
    if (o.fix) {
        o.dist_inv = 1.f / o.dist;
        const float phi_trg = r360m::asinf(o.X * o.dist_inv);
        const float theta_trg = (float)((double)r360m::atan2f_sel(o.Y, o.Z) + R360_PI);
        const float rr = half_nRows - phi_trg * angle_res_inv;
        const float cc = theta_trg * angle_res_inv;
        const int t0 = o.t;
        const bool v0 = o.vis;
        set_pixel(o, rr, cc, true, nRows, nCols);
        o.fix = false;
        changed = o.t != t0 || o.vis != v0;
    }
    return __any(changed);
}

// LUT_xyz_sphere point of a source pixel (:4578-4582), the reference's float expressions
struct Lut3 { float x, y, z; bool valid; };
__device__ __forceinline__ Lut3 lut_point(float d, float sp, float cp, float st, float ct, const IcpConst& C) {
    Lut3 l;
    l.valid = (C.min_d < d && d < C.max_d);
    l.x = d * sp;
    l.y = -d * cp * st;
    l.z = -d * cp * ct;
    return l;
}

// The reference's projection of one LUT point, start to finish (the deferred lanes of the PF 3 loop):
// the transform as written, IEEE sqrt / division, glibc-exact asinf / atan2f, theta + pi in double.
__device__ __forceinline__ Proj project_exact(const Pose12& P, const Lut3& l, float gray_s, int nRows, int nCols,
                                              float half_nRows, float angle_res_inv) {
    Proj o;
    float X = P.R[0] * l.x + P.R[1] * l.y + P.R[2] * l.z; X = X + P.t[0];
    float Y = P.R[3] * l.x + P.R[4] * l.y + P.R[5] * l.z; Y = Y + P.t[1];
    float Z = P.R[6] * l.x + P.R[7] * l.y + P.R[8] * l.z; Z = Z + P.t[2];
    const float dist = sqrtf(X * X + Y * Y + Z * Z);
    const float dist_inv = 1.f / dist;
    const float phi_trg = r360m::asinf(X * dist_inv);
    const float theta_trg = (float)((double)r360m::atan2f_sel(Y, Z) + R360_PI);
    set_pixel(o, half_nRows - phi_trg * angle_res_inv, theta_trg * angle_res_inv, l.valid, nRows, nCols);
    o.X = X; o.Y = Y; o.Z = Z; o.dist = dist; o.dist_inv = dist_inv; o.gray_s = gray_s;
    o.fix = false;
    return o;
}

// PF 3 fast projection (never the final word near a rounding boundary): the reference's p' and |p'|
// (correctly rounded sqrt), then hardware rsq, theta + pi in float, atan2 with one reciprocal, and floor(x + 0.5) rounding
// (= roundf away from the .5 boundaries, which are all inside the guard bands) that shares its
// floor with the guard test.  A lane inside a guard band, or NaN, is flagged in o.fix.
// LEAN (PF 5): p' by three fused multiply-adds per coordinate instead of the reference's six rounded
// operations (|p'| then differs from the reference's by about an ulp; the projection's guard bands are three
// orders of magnitude wider than that, and deferred lanes are re-projected from the exact p').
template <bool LEAN = false>
__device__ __forceinline__ Proj project_fast(const Pose12& P, const Lut3& l, float gray_s, int nRows, int nCols,
                                             float angle_res_inv, float asin_out) {
    Proj o;
    float X, Y, Z;
    if (LEAN) {
        X = __builtin_fmaf(P.R[0], l.x, __builtin_fmaf(P.R[1], l.y, __builtin_fmaf(P.R[2], l.z, P.t[0])));
        Y = __builtin_fmaf(P.R[3], l.x, __builtin_fmaf(P.R[4], l.y, __builtin_fmaf(P.R[5], l.z, P.t[1])));
        Z = __builtin_fmaf(P.R[6], l.x, __builtin_fmaf(P.R[7], l.y, __builtin_fmaf(P.R[8], l.z, P.t[2])));
    } else {
        // p' and |p'| exactly as the reference (they enter the error terms, which steer the GN decisions)
        X = P.R[0] * l.x + P.R[1] * l.y + P.R[2] * l.z; X = X + P.t[0];
        Y = P.R[3] * l.x + P.R[4] * l.y + P.R[5] * l.z; Y = Y + P.t[1];
        Z = P.R[6] * l.x + P.R[7] * l.y + P.R[8] * l.z; Z = Z + P.t[2];
    }
    const float d2 = X * X + Y * Y + Z * Z;
    const float dist_inv = __builtin_amdgcn_rsqf(d2);
    const float phi_trg = r360m::asinf_fast_view(X * dist_inv, asin_out);
    const float theta_trg = r360m::atan2f_fast1(Y, Z) + 3.14159265358979f;
    // u = rr + 0.5, v = cc + 0.5 (half_nRows + 0.5 = nRows / 2 exactly)
    const float u = fmaf(-phi_trg, angle_res_inv, 0.5f * (float)nRows);
    const float v = fmaf(theta_trg, angle_res_inv, 0.5f);
    const float fu = floorf(u), fv = floorf(v);
    const float eu = fabsf(u - fu - 0.5f), ev = fabsf(v - fv - 0.5f);
    o.fix = l.valid && !(eu <= 0.5f - kGuardRow && ev <= 0.5f - kGuardCol);   // NaN -> flagged
    o.vis = l.valid && fu >= 0.f && fu < (float)nRows && fv < (float)nCols;
    o.t = o.vis ? (int)fu * nCols + (int)fv : 0;
    // LEAN: |p'| = d2 rsq(d2) (within ~2 ulp of the correctly rounded root, like the lean error terms it enters)
    o.X = X; o.Y = Y; o.Z = Z; o.dist = LEAN ? d2 * dist_inv : r360m::sqrt_rn(d2); o.dist_inv = dist_inv; o.gray_s = gray_s;
    return o;
}

__device__ __forceinline__ float huber_rn(float e, float reg) {    // weightHuber<float>, bit-exact
    const float a = fabsf(e);
    const float w = r360m::div_rn(r360m::sqrt_rn(2 * reg * a - reg * reg), a);
    return a < reg ? 1.f : w;
}

__device__ __forceinline__ float huber_fast(float e, float reg) {   // weightHuber with hardware sqrt / rcp
    const float a = fabsf(e);
    const float w = __builtin_amdgcn_sqrtf(2 * reg * a - reg * reg) * __builtin_amdgcn_rcpf(a);
    return a < reg ? 1.f : w;
}

// Residuals, weights and Jacobian rows of one projected pixel, accumulated branch-free: a pixel that
// the reference skips contributes through selects that zero its row (never a multiply by 0, which
// would let a NaN of an invalid pixel through).
template <int METHOD, int OCC, bool FAST = false>
__device__ __forceinline__ void contribute(Acc& A, const Proj& o, const float4 G, const float2 T, int fl,
                                           float angle_res_inv, const IcpConst& C) {
#ifdef R360_EXP_NOACC   // experiment builds only: keep the operands alive, skip the math
    A.h[0] += o.vis ? G.x + G.y + G.z + G.w + T.x + T.y + o.X + o.dist : 0.f;
    A.h[28] += o.vis ? 1.f : 0.f;
    return;
#endif
    constexpr bool photo = (METHOD == R360_PHOTO_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    constexpr bool depth = (METHOD == R360_DEPTH_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    const float X = o.X, Y = o.Y, Z = o.Z, dist = o.dist, dist_inv = o.dist_inv;
    // photo saliency fails -> 'continue' skips the depth term too (:3038-3039)
    const bool sal_p = !(fabsf(G.x) < C.thr_int && fabsf(G.y) < C.thr_int);
    const bool sal_d = !(fabsf(G.z) < C.thr_depth && fabsf(G.w) < C.thr_depth);
    const bool fin_d = isfinite(T.y);
    const bool p_ok = photo && o.vis && sal_p;
    const bool d_ok = depth && o.vis && (!photo || sal_p) && fin_d && sal_d;   // (:3064-3073)
    // exact error terms (they steer the accept/reject test :4715)
    // FAST: hardware sqrt / rcp and float products (~1-2 ulp per term; the error and H / g sums keep
    // their fp64 / summation-order tolerances)
    const float photoDiff = T.x - o.gray_s;
    const float whp = FAST ? huber_fast(photoDiff, C.sd_photo) : huberf(photoDiff, C.sd_photo);
    const float wEd = FAST ? whp * C.sd_photo_inv_f * photoDiff
                           : (float)((double)whp * C.sd_photo_inv_d * photoDiff);         // (:2699-2700)
    const float depthDiff = T.y - dist;
    const float sd = C.sd_depth * T.y;
    const float wd = FAST ? huber_fast(depthDiff, sd) * __builtin_amdgcn_rcpf(sd)
                          : huberf(depthDiff, sd) / sd;                                   // (:3077-3078)
    const float wEdep = wd * depthDiff;   // == (float)((double)wd * depthDiff): the f32 product is exact in f64
    // which terms enter the error and which Jacobian rows enter H / g
    bool jp = p_ok, jd = d_ok;
    if (OCC == 0) {
        A.h[28] += o.vis ? 1.f : 0.f;                                               // numVisiblePixels
        if (photo) { A.err2 += p_ok ? (double)(wEd * wEd) : 0.0; A.h[27] += p_ok ? 1.f : 0.f; }
        if (depth) { A.err2 += d_ok ? (double)(wEdep * wEdep) : 0.0; A.h[27] += d_ok ? 1.f : 0.f; }
    } else if (OCC == 1) {
        // errorPhotoICP_sphereOcc1 (:3232-3370): accepted points count, the last accepted one of a
        // target pixel owns its residual; H / g as calcHessGrad_sphere (its Z-buffer never occludes)
        const bool acc = fl & OCC_ACC, own = fl & OCC_OWN;
        A.h[28] += o.vis ? 1.f : 0.f;
        if (photo) { A.err2 += (own && p_ok) ? (double)(wEd * wEd) : 0.0; A.h[27] += (acc && p_ok) ? 1.f : 0.f; }
        if (depth) {
            A.err2d += (own && d_ok) ? (double)(wEdep * wEdep) : 0.0;
            A.h[29] += (acc && d_ok) ? 1.f : 0.f;
        }
    } else {
        // errorPhotoICP_sphereOcc2 (:3720-3855): every accepted point counts and contributes;
        // calcHessGrad_sphereOcc2 (:3861-4250): the last filtered point of a target pixel owns its rows,
        // and a failed depth-saliency test skips the store of both rows
        const bool acc = fl & OCC_ACC, win = fl & OCC_WIN;
        A.h[27] += acc ? 1.f : 0.f;
        if (photo) A.err2 += (acc && p_ok) ? (double)(wEd * wEd) : 0.0;
        if (depth) A.err2d += (acc && d_ok) ? (double)(wEdep * wEdep) : 0.0;
        A.h[28] += win ? 1.f : 0.f;
        jp = win && p_ok && !(depth && fin_d && !sal_d);
        jd = win && d_ok;
    }
    // Jacobian of the spherical warp (:2995-3026), expanded with T36 = [I | -skew(p')]
    float Jw0[6], Jw1[6];
    {
#pragma clang fp contract(fast)
        const float z_inv = __builtin_amdgcn_rcpf(Z);
        const float z_inv2 = z_inv * z_inv;
        const float D_atan = __builtin_amdgcn_rcpf(1 + Y * Y * z_inv2) * angle_res_inv;
        const float P01 = D_atan * z_inv;
        const float P02 = -Y * z_inv2 * D_atan;
        const float x_dist_inv2 = X * (dist_inv * dist_inv);
        const float D_asin = __builtin_amdgcn_rsqf(1 - X * x_dist_inv2) * angle_res_inv;
        const float P10 = -D_asin * dist_inv * (1 - X * x_dist_inv2);
        const float P11 = D_asin * (x_dist_inv2 * Y * dist_inv);
        const float P12 = D_asin * (x_dist_inv2 * Z * dist_inv);
        Jw0[0] = 0.f; Jw0[1] = P01; Jw0[2] = P02; Jw0[3] = P02 * Y - P01 * Z; Jw0[4] = -P02 * X; Jw0[5] = P01 * X;
        Jw1[0] = P10; Jw1[1] = P11; Jw1[2] = P12; Jw1[3] = P12 * Y - P11 * Z; Jw1[4] = P10 * Z - P12 * X;
        Jw1[5] = P11 * X - P10 * Y;
    }
    if (photo) {
#pragma clang fp contract(fast)
        const float w = whp * C.sd_photo_inv_f;                                        // (:3047)
        const float wgx = w * G.x, wgy = w * G.y;
        float J[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) J[k] = jp ? wgx * Jw0[k] + wgy * Jw1[k] : 0.f;
        acc_fma(A, J, jp ? w * photoDiff : 0.f);
    }
    if (depth) {
#pragma clang fp contract(fast)
        // (dgrad * Jw - (p'/|p'|)^T T36): the rotational part of (p'/|p'|)^T T36 is p' x p' / |p'| = 0
        const float js0 = X * dist_inv, js1 = Y * dist_inv, js2 = Z * dist_inv;
        float J[6];
        J[0] = G.z * Jw0[0] + G.w * Jw1[0] - js0;
        J[1] = G.z * Jw0[1] + G.w * Jw1[1] - js1;
        J[2] = G.z * Jw0[2] + G.w * Jw1[2] - js2;
        J[3] = G.z * Jw0[3] + G.w * Jw1[3];
        J[4] = G.z * Jw0[4] + G.w * Jw1[4];
        J[5] = G.z * Jw0[5] + G.w * Jw1[5];
#pragma unroll
        for (int k = 0; k < 6; ++k) J[k] = jd ? wd * J[k] : 0.f;
        acc_fma(A, J, jd ? wd * depthDiff : 0.f);
    }
}

// PF 3's residuals, weights and Jacobian rows: contribute<..>'s terms (exact error terms, fast
// Jacobian) for every occlusion variant, with the skips applied to the weights instead of the rows (a
// lane that contributes nothing has its coordinates replaced by finite ones, so a zero weight zeroes
// its rows exactly) and the counts taken per wave from ballots (SALU).  The depth Huber weight is 1
// for almost every pixel (sigma = 0.2 m per metre of range): its exact sqrt / division run only in
// waves where some lane needs them.
struct WaveCnt { int c27 = 0, c28 = 0, c29 = 0; };

// the ballot of an i1 straight to its SGPR mask (HIP's int __ballot() materialised every predicate as 0 / 1 in a
// VGPR and compared it again: 2 VALU per count)
__device__ __forceinline__ int wave_count(bool b) { return __builtin_popcountll(__builtin_amdgcn_ballot_w64(b)); }

template <int METHOD, int OCC>
__device__ __forceinline__ void contribute_fast(Acc& A, WaveCnt& W, const Proj& o, const float4 G, const float2 T,
                                                int fl, float angle_res_inv, const IcpConst& C) {
#ifdef R360_EXP_NOACC   // experiment builds only: keep the operands alive, skip the math
    A.h[0] += o.vis ? G.x + G.y + G.z + G.w + T.x + T.y + o.X + o.dist : 0.f;
    W.c28 += wave_count(o.vis);
    return;
#endif
    constexpr bool photo = (METHOD == R360_PHOTO_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    constexpr bool depth = (METHOD == R360_DEPTH_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    const bool sal_p = !(fabsf(G.x) < C.thr_int && fabsf(G.y) < C.thr_int);
    const bool sal_d = !(fabsf(G.z) < C.thr_depth && fabsf(G.w) < C.thr_depth);
    const bool fin_d = isfinite(T.y);
    const bool p_ok = photo && o.vis && sal_p;
    const bool d_ok = depth && o.vis && (!photo || sal_p) && fin_d && sal_d;   // (:3064-3073)
    // error terms exactly as the reference's (correctly rounded sqrt / division, no contraction): they
    // steer the GN accept / stop decisions, which must not flip on a rounding difference
    const float photoDiff = T.x - o.gray_s;
    const float whp = huber_rn(photoDiff, C.sd_photo);
    const float wEd = (float)((double)whp * C.sd_photo_inv_d * photoDiff);                 // (:2699-2700)
    const float depthDiff = T.y - o.dist;
    const float sd = C.sd_depth * T.y;
    float hd = 1.f;
    if (__any(d_ok && !(fabsf(depthDiff) < sd))) hd = huber_rn(depthDiff, sd);
    const float wd_ = r360m::div_rn(hd, sd);                                               // (:3077-3078)
    const float wEdep = wd_ * depthDiff;   // == (float)((double)wd * depthDiff)
    const float ep = wEd * wEd, ed = wEdep * wEdep;
    bool jp = p_ok, jd = d_ok;
    if (OCC == 0) {
        W.c28 += wave_count(o.vis);                                                        // numVisiblePixels
        W.c27 += (photo ? wave_count(p_ok) : 0) + (depth ? wave_count(d_ok) : 0);
        // one f64 add per pixel: the pixel's two squared terms are summed in f32 first (2^-24 relative per
        // pixel, far below the accept test's resolution; the summation order differs from the
        // reference's OpenMP reduction anyway)
        A.err2 += (double)((p_ok ? ep : 0.f) + (d_ok ? ed : 0.f));
    } else if (OCC == 1) {
        // errorPhotoICP_sphereOcc1 (:3232-3370): accepted points count, the last accepted one of a target
        // pixel owns its residual; H / g as calcHessGrad_sphere (its Z-buffer never occludes)
        const bool acc = fl & OCC_ACC, own = fl & OCC_OWN;
        W.c28 += wave_count(o.vis);
        if (photo) { A.err2 += (own && p_ok) ? (double)ep : 0.0; W.c27 += wave_count(acc && p_ok); }
        if (depth) { A.err2d += (own && d_ok) ? (double)ed : 0.0; W.c29 += wave_count(acc && d_ok); }
    } else {
        // errorPhotoICP_sphereOcc2 (:3720-3855): every accepted point counts and contributes;
        // calcHessGrad_sphereOcc2 (:3861-4250): the last filtered point of a target pixel owns its rows,
        // and a failed depth-saliency test skips the store of both rows
        const bool acc = fl & OCC_ACC, win = fl & OCC_WIN;
        W.c27 += wave_count(acc);
        if (photo) A.err2 += (acc && p_ok) ? (double)ep : 0.0;
        if (depth) A.err2d += (acc && d_ok) ? (double)ed : 0.0;
        W.c28 += wave_count(win);
        jp = win && p_ok && !(depth && fin_d && !sal_d);
        jd = win && d_ok;
    }
    const float wp = jp ? whp * C.sd_photo_inv_f : 0.f;                                    // (:3047)
    const float rp = wp * photoDiff;
    const float wd = jd ? wd_ : 0.f;
    const float rd = jd ? wEdep : 0.f;   // |p'| of a lane without a point can be NaN
    const float X = o.vis ? o.X : 1.f, Y = o.vis ? o.Y : 1.f, Z = o.vis ? o.Z : 1.f;
    const float dist_inv = o.vis ? o.dist_inv : 0.5f;
    {
#pragma clang fp contract(fast)
        // Jacobian of the spherical warp (:2995-3026): row = [gx gy] J_proj [I | -skew(p')] = [u, p' x u]
        // with u = J_proj^T [gx gy]^T (the 3-vector of the translation part; u^T (-skew(p')) = (p' x u)^T).
        // J_proj in closed form, with r2 = Y^2 + Z^2, d2 = |p'|^2 and a = 1 / angle_res:
        //   theta row (0, a Z / r2, -a Y / r2);  phi row (-a r2 / (sqrt(r2) d2), a X Y / (sqrt(r2) d2),
        //   a X Z / (sqrt(r2) d2)) — the reference's D_atan / D_asin products (:3000-3016) simplified.
        const float r2 = Y * Y + Z * Z;
        const float s = __builtin_amdgcn_rcpf(r2) * angle_res_inv;                        // theta row scale
        const float t = __builtin_amdgcn_rsqf(r2) * (dist_inv * dist_inv) * angle_res_inv; // phi row scale
        auto row = [&](float gx, float gy, float& u0, float& u1, float& u2) {
            const float A = gx * s, B = gy * t, BX = B * X;
            u0 = -B * r2;
            u1 = A * Z + BX * Y;
            u2 = BX * Z - A * Y;
        };
        auto acc_row = [&](float u0, float u1, float u2, float r) {
            const float J[6] = {u0, u1, u2, Y * u2 - Z * u1, Z * u0 - X * u2, X * u1 - Y * u0};
            acc_fma(A, J, r);
        };
        if (photo) {
            float u0, u1, u2;
            row(wp * G.x, wp * G.y, u0, u1, u2);
            acc_row(u0, u1, u2, rp);
        }
        if (depth) {
            // (dgrad * J_w - (p'/|p'|)^T T36): the rotational part of (p'/|p'|)^T T36 is p' x p' / |p'| = 0,
            // so the unit-vector term enters u only
            float u0, u1, u2;
            row(wd * G.z, wd * G.w, u0, u1, u2);
            const float wdi = wd * dist_inv;
            acc_row(u0 - wdi * X, u1 - wdi * Y, u2 - wdi * Z, rd);
        }
    }
}

// PF 5's residuals, weights and Jacobian rows (plain pass, OCC 0): contribute_fast with the error terms in
// fast single precision instead of the reference's exact float / double mix.
//  * Huber weights without a square root or a division: for |e| >= k, sqrt(2 k |e| - k^2) / |e| = t rsq(t e^2)
//    with t = 2 k |e| - k^2; the depth weight's 1 / sigma folds into the same reciprocal square root
//    (w_d = rsq(sigma^2) below sigma, t rsq(t e^2 sigma^2) above).  One hardware rsq per term (~1 ulp)
//    replaces sqrt_rn + div_rn (photo), div_rn and a wave-wide exact Huber branch (depth).
//  * Photo residual w e / sigma in float (the reference's double product, :2699-2700, rounds to float anyway).
//  * The squared residuals are summed per lane in float and in double across lanes and workgroups (~1e-7
//    relative; the error value's bar is 1e-5).
// The weights are continuous at |e| = k (both branches give 1), so the comparison needs no guard band.
// FIN = false: the target depth is known finite (PF 6 unpacks it from the packed image's millimetres).
template <int METHOD, bool FIN = true>
__device__ __forceinline__ void contribute_lean(Acc& A, WaveCnt& W, float& errf, const Proj& o, const float4 G,
                                                const float2 T, float angle_res_inv, const IcpConst& C) {
    constexpr bool photo = (METHOD == R360_PHOTO_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    constexpr bool depth = (METHOD == R360_DEPTH_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    const bool sal_p = !(fabsf(G.x) < C.thr_int && fabsf(G.y) < C.thr_int);
    const bool sal_d = !(fabsf(G.z) < C.thr_depth && fabsf(G.w) < C.thr_depth);
    const bool fin_d = !FIN || isfinite(T.y);
    const bool p_ok = photo && o.vis && sal_p;
    const bool d_ok = depth && o.vis && (!photo || sal_p) && fin_d && sal_d;   // (:3064-3073)
    float wp = 0.f, rp = 0.f, wd = 0.f, rd = 0.f;
    {
#pragma clang fp contract(fast)
        if (photo) {
            const float e = T.x - o.gray_s;
            const float a = fabsf(e), k = C.sd_photo;
            const float t = 2.f * k * a - k * k;
            const float h = a < k ? 1.f : t * __builtin_amdgcn_rsqf(t * a * a);   // weightHuber (:545-554)
            wp = p_ok ? h * C.sd_photo_inv_f : 0.f;                                 // (:3047)
            rp = wp * e;
        }
        if (depth) {
            const float e = T.y - o.dist;
            const float a = fabsf(e), k = C.sd_depth * T.y, k2 = k * k;
            const float t = 2.f * k * a - k2;
            const bool in = a < k;
            const float w = (in ? 1.f : t) * __builtin_amdgcn_rsqf(in ? k2 : t * a * a * k2);   // (:3077-3078)
            wd = d_ok ? w : 0.f;
            rd = d_ok ? w * e : 0.f;   // |p'| of a lane without a point can be NaN
        }
        errf += rp * rp + rd * rd;
    }
    W.c28 += wave_count(o.vis);                                                            // numVisiblePixels
    W.c27 += (photo ? wave_count(p_ok) : 0) + (depth ? wave_count(d_ok) : 0);
    // p' of a lane without a point is finite (a LUT point, transformed), but r2 and |p'| may be 0 there: the lane's
    // zero weights must not meet an infinite scale
    const float X = o.X, Y = o.Y, Z = o.Z;
    const float dist_inv = o.vis ? o.dist_inv : 0.5f;
    {
#pragma clang fp contract(fast)
        // the closed-form Jacobian rows of contribute_fast: row = [u, p' x u], u = J_proj^T [gx gy]^T
        const float r2 = o.vis ? Y * Y + Z * Z : 1.f;
        const float s = __builtin_amdgcn_rcpf(r2) * angle_res_inv;
        const float t = __builtin_amdgcn_rsqf(r2) * (dist_inv * dist_inv) * angle_res_inv;
        auto row = [&](float gx, float gy, float& u0, float& u1, float& u2) {
            const float A = gx * s, B = gy * t, BX = B * X;
            u0 = -B * r2;
            u1 = A * Z + BX * Y;
            u2 = BX * Z - A * Y;
        };
        auto acc_row = [&](float u0, float u1, float u2, float r) {
            const float J[6] = {u0, u1, u2, Y * u2 - Z * u1, Z * u0 - X * u2, X * u1 - Y * u0};
            acc_fma(A, J, r);
        };
        if (photo) {
            float u0, u1, u2;
            row(wp * G.x, wp * G.y, u0, u1, u2);
            acc_row(u0, u1, u2, rp);
        }
        if (depth) {
            float u0, u1, u2;
            row(wd * G.z, wd * G.w, u0, u1, u2);
            const float wdi = wd * dist_inv;
            acc_row(u0 - wdi * X, u1 - wdi * Y, u2 - wdi * Z, rd);
        }
    }
}

#if R360_PK_ACC
// Packed accumulation (PF 6): the 27 sums of J J^T and J r over a lane's pixels as 12 register pairs and 3 scalars,
// updated by v_pk_fma_f32 (two FMAs per VALU instruction) instead of 27 v_fma per Jacobian row.  The row's
// components are taken in the order q = (u1, u2 | u0, J3 | J4, J5 | r) and summed two rows of H at a time: pair
// (q0, q1) times every q_j, j >= 1, and so on; the broadcast operand of each update comes from a half of an
// existing pair (op_sel), so the update needs no register moves.  pk_fold maps the sums back to Acc's slots.
typedef float f2v __attribute__((ext_vector_type(2)));
struct AccPk {
    f2v a0, a2, a3, a4, a5, a6;   // (q0 q0, q1 q1), (q0, q1) x q2 .. q6
    f2v b0, b4, b5, b6;           // (q2 q2, q3 q3), (q2, q3) x q4 .. q6
    f2v c0, c6;                   // (q4 q4, q5 q5), (q4, q5) x q6
    float sa, sb, sc;             // q0 q1, q2 q3, q4 q5
};
__device__ __forceinline__ f2v pkfma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2v bc2(float x) { return f2v{x, x}; }

__device__ __forceinline__ void pk_zero(AccPk& K) {
    K.a0 = K.a2 = K.a3 = K.a4 = K.a5 = K.a6 = K.b0 = K.b4 = K.b5 = K.b6 = K.c0 = K.c6 = f2v{0.f, 0.f};
    K.sa = K.sb = K.sc = 0.f;
}

// one Jacobian row J = [u0, u1, u2, p' x u] (u12 = (u1, u2)) with residual r
__device__ __forceinline__ void pk_row(AccPk& K, f2v u12, float u0, float X, float Y, float Z, float r) {
#pragma clang fp contract(fast)
    const float J3 = Y * u12.y - Z * u12.x, J4 = Z * u0 - X * u12.y, J5 = X * u12.x - Y * u0;
    const f2v Pb = f2v{u0, J3}, Pc = f2v{J4, J5};
    K.a0 = pkfma(u12, u12, K.a0);
    K.sa = __builtin_fmaf(u12.x, u12.y, K.sa);
    K.a2 = pkfma(u12, bc2(u0), K.a2);
    K.a3 = pkfma(u12, bc2(J3), K.a3);
    K.a4 = pkfma(u12, bc2(J4), K.a4);
    K.a5 = pkfma(u12, bc2(J5), K.a5);
    K.a6 = pkfma(u12, bc2(r), K.a6);
    K.b0 = pkfma(Pb, Pb, K.b0);
    K.sb = __builtin_fmaf(u0, J3, K.sb);
    K.b4 = pkfma(Pb, bc2(J4), K.b4);
    K.b5 = pkfma(Pb, bc2(J5), K.b5);
    K.b6 = pkfma(Pb, bc2(r), K.b6);
    K.c0 = pkfma(Pc, Pc, K.c0);
    K.sc = __builtin_fmaf(J4, J5, K.sc);
    K.c6 = pkfma(Pc, bc2(r), K.c6);
}

// the packed sums into Acc's slots (0..20 upper-triangle H row-major, 21..26 g)
__device__ __forceinline__ void pk_fold(Acc& A, const AccPk& K) {
    A.h[6] += K.a0.x;  A.h[11] += K.a0.y; A.h[7] += K.sa;
    A.h[1] += K.a2.x;  A.h[2] += K.a2.y;
    A.h[8] += K.a3.x;  A.h[12] += K.a3.y;
    A.h[9] += K.a4.x;  A.h[13] += K.a4.y;
    A.h[10] += K.a5.x; A.h[14] += K.a5.y;
    A.h[22] += K.a6.x; A.h[23] += K.a6.y;
    A.h[0] += K.b0.x;  A.h[15] += K.b0.y; A.h[3] += K.sb;
    A.h[4] += K.b4.x;  A.h[16] += K.b4.y;
    A.h[5] += K.b5.x;  A.h[17] += K.b5.y;
    A.h[21] += K.b6.x; A.h[24] += K.b6.y;
    A.h[18] += K.c0.x; A.h[20] += K.c0.y; A.h[19] += K.sc;
    A.h[25] += K.c6.x; A.h[26] += K.c6.y;
}

// contribute_lean<METHOD, false> (PF 6: the target depth is finite) with the Jacobian rows built in pairs and summed
// by pk_row: u = J_proj^T [gx gy]^T as (A, B) = w (gx, gy) * (s, t), u0 = -B r2, (u1, u2) = A (Z, -Y) + B X (Y, Z)
template <int METHOD>
__device__ __forceinline__ void contribute_pk(AccPk& K, WaveCnt& W, float& errf, const Proj& o, const float4 G,
                                              const float2 T, float angle_res_inv, const IcpConst& C) {
    constexpr bool photo = (METHOD == R360_PHOTO_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    constexpr bool depth = (METHOD == R360_DEPTH_CONSISTENCY || METHOD == R360_PHOTO_DEPTH);
    const bool sal_p = !(fabsf(G.x) < C.thr_int && fabsf(G.y) < C.thr_int);
    const bool sal_d = !(fabsf(G.z) < C.thr_depth && fabsf(G.w) < C.thr_depth);
    const bool p_ok = photo && o.vis && sal_p;
    const bool d_ok = depth && o.vis && (!photo || sal_p) && sal_d;   // (:3064-3073)
    float wp = 0.f, rp = 0.f, wd = 0.f, rd = 0.f;
    {
#pragma clang fp contract(fast)
        if (photo) {
            const float e = T.x - o.gray_s;
            const float a = fabsf(e), k = C.sd_photo;
            const float t = 2.f * k * a - k * k;
            const float h = a < k ? 1.f : t * __builtin_amdgcn_rsqf(t * a * a);   // weightHuber (:545-554)
            wp = p_ok ? h * C.sd_photo_inv_f : 0.f;                                 // (:3047)
            rp = wp * e;
        }
        if (depth) {
            const float e = T.y - o.dist;
            const float a = fabsf(e), k = C.sd_depth * T.y, k2 = k * k;
            const float t = 2.f * k * a - k2;
            const bool in = a < k;
            const float w = (in ? 1.f : t) * __builtin_amdgcn_rsqf(in ? k2 : t * a * a * k2);   // (:3077-3078)
            wd = d_ok ? w : 0.f;
            rd = d_ok ? w * e : 0.f;
        }
        errf += rp * rp + rd * rd;
    }
    W.c28 += wave_count(o.vis);                                                            // numVisiblePixels
    W.c27 += (photo ? wave_count(p_ok) : 0) + (depth ? wave_count(d_ok) : 0);
    const float X = o.X, Y = o.Y, Z = o.Z;
    const float dist_inv = o.vis ? o.dist_inv : 0.5f;
    {
#pragma clang fp contract(fast)
        const float r2 = o.vis ? Y * Y + Z * Z : 1.f;
        // 1 / angle_res enters through the row's weight (no loop-invariant register pair)
        const f2v st = f2v{__builtin_amdgcn_rcpf(r2), __builtin_amdgcn_rsqf(r2) * (dist_inv * dist_inv)};
        const f2v YZ = f2v{Y, Z}, ZnY = f2v{Z, -Y};
        auto row = [&](f2v g, float w, f2v& u12, float& u0) {
            const f2v AB = (g * st) * bc2(w * angle_res_inv);
            const float BX = AB.y * X;
            u0 = -AB.y * r2;
            u12 = pkfma(bc2(BX), YZ, bc2(AB.x) * ZnY);
        };
        if (photo) {
            f2v u12;
            float u0;
            row(f2v{G.x, G.y}, wp, u12, u0);
            pk_row(K, u12, u0, X, Y, Z, rp);
        }
        if (depth) {
            f2v u12;
            float u0;
            row(f2v{G.z, G.w}, wd, u12, u0);
            const float wdi = wd * dist_inv;
            pk_row(K, pkfma(bc2(-wdi), YZ, u12), u0 - wdi * X, X, Y, Z, rd);
        }
    }
}
#endif

// ---------------------------------------------------------------- GN step (thread 0 of last block)
#include "icp_gn.inc"


// The last arrival of a pass's jobs (a job's last workgroup, or block 0 of a job that exits at entry) closes
// the pass's in-kernel execution span, if any job ran.  kp (optional): kt[0] and the level's three accumulators,
// loaded before the step (nothing writes them during a launch but its last arrival).  A one-job launch needs no
// arrival count: its job's last workgroup is the last arrival, and the span is stored without a dependent
// memory round trip behind the step (three of them were ~2 us of every lone pass's tail).
__device__ __forceinline__ void pass_arrive(unsigned long long* kt, bool ran, int level,
                                            const unsigned long long* kp = nullptr, bool persist = false) {
    unsigned long long runs = ran ? 1ull : 0ull;
    if (gridDim.y > 1) {
        const unsigned long long prev = __hip_atomic_fetch_add(kt + 17, 1ull + (ran ? (1ull << 32) : 0ull),
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)prev != gridDim.y - 1) return;
        __hip_atomic_store(kt + 17, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        runs += prev >> 32;
    }
    if (runs == 0) return;
    const int lv = level & 7;
    const unsigned long long t0 = kp ? kp[0] : __hip_atomic_load(kt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long a = kp ? kp[1] : kt[1 + lv], b = kp ? kp[2] : kt[9 + lv], c = kp ? kp[3] : kt[18 + lv];
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    // sc1 stores: in a persistent launch the next pass's last workgroup (another CU) reads them
    __hip_atomic_store(kt + 1 + lv, a + (t1 > t0 ? t1 - t0 : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(kt + 9 + lv, b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(kt + 18 + lv, c + runs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // job passes (pairs) the launch ran
    if (persist) __hip_atomic_store(kt, t1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // the next pass's start
}

// TOP = 1 only renames the level-0 instantiation, so traces (rocprofv3) separate level 0 from level 1,
// which launch the same grid.  One launch runs gridDim.y independent alignments (jobs.j[blockIdx.y]), each
// on gridDim.x workgroups with its own records, tickets and GN state: a job's sums and step are exactly
// those of the same job launched alone.
// One pass of one workgroup (the kernels below): PASS_SKIPPED if the job had stopped (nothing done),
// PASS_STEPPED in the job's last workgroup (it ran the GN step and wrote the state back), PASS_ARRIVED otherwise.
// PERSIST: the pass inside the persistent level launch (k_icp_level), where the state was written during the
// launch by another workgroup: every load of it is an sc1 (L1-bypassing) vector load and the write-back is sc1
// stores drained before the hand-off (MI355X_MICROARCH.md 'Valid forms', row 1).
enum : int { PASS_SKIPPED = 0, PASS_ARRIVED = 1, PASS_STEPPED = 2 };
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int ld_sc1_i(const int* p) {
    return (int)__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1_f(const float* p) {
    return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <int METHOD, int PF, int TOP, int OCC, bool PERSIST>
__device__ __forceinline__ int icp_pass_body(const IcpJobs& jobs, const float* __restrict__ sinphi,
                                             const float* __restrict__ cosphi, const float* __restrict__ sinth,
                                             const float* __restrict__ costh, int nRows, int nCols,
                                             const IcpConst& C, int first, int eval_only,
                                             unsigned long long* __restrict__ kt,
                                             const uint8_t* __restrict__ occf, const int tidx, const int bidx) {
    __shared__ float s_red[NW][32];
    __shared__ double s_err[NW], s_errd[NW];
    __shared__ double s_fin[RG][32];
#if !R360_POLL
    __shared__ int s_last;
#endif
    __shared__ int s_qn[NW];   // PF 5: deferred entries per wave
    __shared__ GnShared s_gn;
    __shared__ IcpState s_state;

    const IcpJob& J = jobs.j[blockIdx.y];
    const float2* __restrict__ src = J.src;
    const float2* __restrict__ trg = J.trg;
    const float4* __restrict__ tg = J.tg;
    const float4* __restrict__ pts = J.pts;
    const int* __restrict__ npts = J.npts;
    IcpState* S = J.S;
    double* __restrict__ partials = J.partials;
    unsigned* __restrict__ gcnt = J.gcnt;
    int* __restrict__ dq = J.dq;

    // execution span: the start of the launch's first workgroup (dispatched first).  One store, not an
    // atomic-min per workgroup: same-address atomics serialise at the memory side (~25 ns each), and 512
    // of them outlasted a short pass.
    // (persistent launch: at its first pass; a later pass starts where the previous one's step published)
    if (bidx == 0 && blockIdx.y == 0 && tidx == 0 && (!PERSIST || first))
        __hip_atomic_store(kt, (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
#ifdef R360_STAMPS
    // R360_STAMP_ENTRY: the start stamp before the state read (default: after it)
#ifdef R360_STAMP_ENTRY
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
#endif
    // Persistent launch: 18 lanes of the workgroup read the state words once (sc1) and hand them over in LDS.  Every
    // wave reading them itself put 2048 waves x 18 loads of the same two lines on one L2 channel per XCD at every
    // pass start (~3 us; the per-pass kernel reads them through the scalar cache).
    __shared__ unsigned s_pst[18];   // pose (16), stop, active
    if constexpr (PERSIST) {
        const float* pm0 = first ? S->pose : S->cand;
        if (tidx < 16) s_pst[tidx] = __float_as_uint(ld_sc1_f(pm0 + tidx));
        else if (tidx == 16) s_pst[16] = (unsigned)ld_sc1_i(&S->stop);
        else if (tidx == 17) s_pst[17] = (unsigned)ld_sc1_i(&S->active);
        __syncthreads();
    }
    const int st_stop = PERSIST ? (int)__builtin_amdgcn_readfirstlane(s_pst[16]) : S->stop;
    const int st_active = PERSIST ? (int)__builtin_amdgcn_readfirstlane(s_pst[17]) : S->active;
    if (st_stop || (!first && !st_active && !eval_only)) {
        if (!PERSIST && bidx == 0 && tidx == 0) pass_arrive(kt, false, C.level);
        return PASS_SKIPPED;
    }
#if defined(R360_STAMPS) && !defined(R360_STAMP_ENTRY)
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif

    const float* pm = (first && !eval_only) ? S->pose : S->cand;
    Pose12 P;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
            P.R[r * 3 + c] = PERSIST ? __uint_as_float(__builtin_amdgcn_readfirstlane(s_pst[c * 4 + r])) : pm[c * 4 + r];
        P.t[r] = PERSIST ? __uint_as_float(__builtin_amdgcn_readfirstlane(s_pst[12 + r])) : pm[12 + r];
    }
    const float angle_res = (float)(2 * R360_PI / nCols);
    const float angle_res_inv = 1 / angle_res;
    const float half_nRows = (float)(0.5 * nRows - 0.5);
    const float asin_out = asin_out_for(nRows, nCols);

    Acc A;
#pragma unroll
    for (int k = 0; k < 32; ++k) A.h[k] = 0.f;
    A.err2 = 0.0;
    A.err2d = 0.0;
    auto flag = [&](int i) { return OCC ? (int)occf[i] : 0; };
    WaveCnt W;   // PF 3: wave-uniform counts
    float errf = 0.f;   // PF 5: the lane's squared residuals in float

    const int units = (nRows * nCols) >> 2;  // 4 pixels of one row per unit (nCols % 4 == 0)
    const float4* src4 = reinterpret_cast<const float4*>(src);
    const float4* st4 = reinterpret_cast<const float4*>(sinth);
    const float4* ct4 = reinterpret_cast<const float4*>(costh);
    const int cq = nCols >> 2;
    auto one = [&](float d, float g, float sp, float cp, float st, float ct, int fl) {
        Proj o = project(P, d, g, sp, cp, st, ct, nRows, nCols, half_nRows, angle_res_inv, C);
        project_fix(o, nRows, nCols, half_nRows, angle_res_inv);
        const float4 G = tg[o.t];
        const float2 T = trg[o.t];
        contribute<METHOD, OCC>(A, o, G, T, fl, angle_res_inv, C);
    };
    auto two = [&](float d0, float g0, float d1, float g1, float sp, float cp, float st0, float ct0, float st1,
                   float ct1, int fl0, int fl1) {
        // project both, issue both gathers, then the math (ILP + loads in flight)
        Proj o0 = project(P, d0, g0, sp, cp, st0, ct0, nRows, nCols, half_nRows, angle_res_inv, C);
        Proj o1 = project(P, d1, g1, sp, cp, st1, ct1, nRows, nCols, half_nRows, angle_res_inv, C);
        project_fix(o0, nRows, nCols, half_nRows, angle_res_inv);
        project_fix(o1, nRows, nCols, half_nRows, angle_res_inv);
        const float4 G0 = tg[o0.t], G1 = tg[o1.t];
        const float2 T0 = trg[o0.t], T1 = trg[o1.t];
        contribute<METHOD, OCC>(A, o0, G0, T0, fl0, angle_res_inv, C);
        contribute<METHOD, OCC>(A, o1, G1, T1, fl1, angle_res_inv, C);
    };
    const int stride = gridDim.x * TPB;
    if (PF == 1) {
        // large levels: 4-pixel units (vector loads), processed as two pixel pairs (ILP)
        for (int u = bidx * TPB + tidx; u < units; u += stride) {
            const int r = u / cq;
            const int c4 = u - r * cq;
            const float4 a = src4[2 * u], b = src4[2 * u + 1];  // {g0,d0,g1,d1} {g2,d2,g3,d3}
            const float4 s = st4[c4], c = ct4[c4];
            const float sp = sinphi[r], cp = cosphi[r];
            two(a.y, a.x, a.w, a.z, sp, cp, s.x, c.x, s.y, c.y, flag(4 * u), flag(4 * u + 1));
            two(b.y, b.x, b.w, b.z, sp, cp, s.z, c.z, s.w, c.w, flag(4 * u + 2), flag(4 * u + 3));
        }
    } else if (PF == 2) {
        // software-pipelined pixel stream, one wave = 64 consecutive pixels of one row (nCols % 64 == 0,
        // so row/column come from wave-uniform scalar arithmetic and the row LUT is wave-uniform): while
        // chunk k is accumulated, chunk k+1's target gathers and chunk k+2's source loads are in flight
        const int npx = nRows * nCols;
        const int lane = tidx & 63;
        struct Src { float d, g, sp, cp, st, ct; int f; };
        auto ld = [&](int base) {                          // base: wave-uniform first pixel
            const int r = __builtin_amdgcn_readfirstlane(base / nCols);
            const int c = base - r * nCols + lane;
            const float2 a = src[base + lane];
            return Src{a.y, a.x, sinphi[r], cosphi[r], sinth[c], costh[c], flag(base + lane)};
        };
        const Gather gt{__builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(tg), 0, npx * 16, 0x00020000),
                        __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(trg), 0, npx * 8, 0x00020000)};
        const int b0 = __builtin_amdgcn_readfirstlane((bidx * TPB + (tidx & ~63)));
        if (b0 < npx) {
            // Unrolled by two with fixed register roles (A, B) and unconditional loads (the chunk index is
            // clamped to the wave's last chunk): no loop-carried copies of in-flight loads and the same
            // number of loads on every path, so each wait names exactly the loads it needs.
            const int n_it = (npx - 1 - b0) / stride + 1;  // chunks of this wave (>= 1)
            auto base = [&](int k) { return b0 + (k < n_it ? k : n_it - 1) * stride; };
            auto prj = [&](const Src& x) {
                return project(P, x.d, x.g, x.sp, x.cp, x.st, x.ct, nRows, nCols, half_nRows, angle_res_inv, C);
            };
            // Per half-iteration h: load the source of chunk h+2, project chunk h+1 and issue its gathers,
            // accumulate chunk h.  Loads are issued in the order they are consumed, so the in-order
            // vmcnt lets each wait skip the five younger loads still in flight.
            // The gathers of a chunk are issued speculatively from the fast projection; the rare
            // guard-band lanes are re-projected at the next half-iteration boundary and, if a pixel
            // changed, the chunk's gathers are re-issued before it is accumulated.
            Src sA = ld(base(0));
            Src sB = ld(base(1));
            Proj oA = prj(sA);
            int fA = sA.f;
            project_fix(oA, nRows, nCols, half_nRows, angle_res_inv);
            float4 GA = gt.g(oA.t);
            float2 TA = gt.T(oA.t);
            for (int k = 0;; k += 2) {
                sA = ld(base(k + 2));
                Proj oB = prj(sB);
                const int fB = sB.f;
                float4 GB = gt.g(oB.t);
                float2 TB = gt.T(oB.t);
                contribute<METHOD, OCC>(A, oA, GA, TA, fA, angle_res_inv, C);
                if (k + 1 >= n_it) break;
                if (project_fix(oB, nRows, nCols, half_nRows, angle_res_inv)) { GB = gt.g(oB.t); TB = gt.T(oB.t); }
                sB = ld(base(k + 3));
                oA = prj(sA);
                fA = sA.f;
                GA = gt.g(oA.t);
                TA = gt.T(oA.t);
                contribute<METHOD, OCC>(A, oB, GB, TB, fB, angle_res_inv, C);
                if (k + 2 >= n_it) break;
                if (project_fix(oA, nRows, nCols, half_nRows, angle_res_inv)) { GA = gt.g(oA.t); TA = gt.T(oA.t); }
            }
        }
    } else if (PF == 3) {
        // PF 2's pipelined wave stream with the guard-band lanes DEFERRED instead of fixed in place: a
        // lane whose fast projection lands near a rounding boundary drops out of its chunk (no
        // contribution) and its pixel index goes to the wave's queue in global memory (room for every
        // pixel of the wave, so it never overflows); after the stream the wave runs the exact
        // projection (project_exact) over its queue, 64 pixels at a time.  The chunk loop keeps one
        // straight-line path (no re-issued gathers, no conditional accumulation that would make the
        // compiler copy the accumulators), and the exact code runs at full lane occupancy instead of
        // once per chunk that has any flagged lane (about a quarter of them at level 0).
        const int npx = nRows * nCols;
        const int lane = tidx & 63;
        const int qcap = ((npx + stride - 1) / stride) * 64;
        int* q = dq + ((long)bidx * NW + (tidx >> 6)) * qcap;
        int qn = 0;   // wave-uniform queue length
        auto acc = [&](const Proj& o, const float4 G, const float2 T, int fl) {
            contribute_fast<METHOD, OCC>(A, W, o, G, T, fl, angle_res_inv, C);
        };
        struct Src { float d, g, sp, cp, st, ct; int f; };
        auto ld = [&](int base) {
            const int r = __builtin_amdgcn_readfirstlane(base / nCols);
            const int c = base - r * nCols + lane;
            const float2 a = src[base + lane];
            return Src{a.y, a.x, sinphi[r], cosphi[r], sinth[c], costh[c], flag(base + lane)};
        };
        const Gather gt{__builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(tg), 0, npx * 16, 0x00020000),
                        __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(trg), 0, npx * 8, 0x00020000)};
        auto prj = [&](const Src& x) {
            return project_fast(P, lut_point(x.d, x.sp, x.cp, x.st, x.ct, C), x.g, nRows, nCols, angle_res_inv, asin_out);
        };
        // queue the flagged lanes of a chunk and take them out of it
        auto defer = [&](Proj& o, int& fl, int base) {
            const unsigned long long m = __ballot(o.fix);
            if (m) {
                const int pos = qn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                if (o.fix) { q[pos] = base + lane; o.vis = false; o.t = 0; fl = 0; }   // Occ2 counts read the flags
                qn += __popcll(m);
            }
        };
        const int b0 = __builtin_amdgcn_readfirstlane((bidx * TPB + (tidx & ~63)));
#ifdef R360_EXP_NOLOOP   // experiment builds only: the pass without its pixel loop (fixed costs)
        if (false) {
#else
        if (b0 < npx) {
#endif
            const int n_it = (npx - 1 - b0) / stride + 1;
            auto base = [&](int k) { return b0 + (k < n_it ? k : n_it - 1) * stride; };
            Src sA = ld(base(0));
            Src sB = ld(base(1));
            Proj oA = prj(sA);
            int fA = sA.f;
            defer(oA, fA, base(0));
            float4 GA = gt.g(oA.t);
            float2 TA = gt.T(oA.t);
            for (int k = 0;; k += 2) {
                sA = ld(base(k + 2));
                Proj oB = prj(sB);
                int fB = sB.f;
                if (k + 1 < n_it) defer(oB, fB, base(k + 1));   // a clamped tail chunk is never accumulated
                const float4 GB = gt.g(oB.t);
                const float2 TB = gt.T(oB.t);
                acc(oA, GA, TA, fA);
                if (k + 1 >= n_it) break;
                sB = ld(base(k + 3));
                oA = prj(sA);
                fA = sA.f;
                if (k + 2 < n_it) defer(oA, fA, base(k + 2));
                GA = gt.g(oA.t);
                TA = gt.T(oA.t);
                acc(oB, GB, TB, fB);
                if (k + 2 >= n_it) break;
            }
        }
#ifdef R360_EXP_NODRAIN   // experiment builds only: deferred lanes dropped
        qn = 0;
#endif
        if (qn > 0) {
            // the queue was written by other lanes of this wave: order those stores before the reads
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            for (int s0 = 0; s0 < qn; s0 += 64) {
                const bool act = s0 + lane < qn;
                const int i = act ? q[s0 + lane] : 0;
                const int r = i / nCols, c = i - r * nCols;
                const float2 a = src[i];
                Proj o = project_exact(P, lut_point(a.y, sinphi[r], cosphi[r], sinth[c], costh[c], C), a.x, nRows,
                                       nCols, half_nRows, angle_res_inv);
                o.vis = o.vis && act;
                o.t = o.vis ? o.t : 0;
                acc(o, gt.g(o.t), gt.T(o.t), act ? flag(i) : 0);
            }
        }
    } else if (PF == 4 || PF == 5) {
        // PF 3's wave stream over the level's COMPACTED source points (LevelBufs::pts, built once per frame):
        // only pixels with minDepth < depth < maxDepth, as {LUT point, gray}, in raster order.  No row/column
        // tables, no LUT arithmetic and no lanes spent on pixels without depth.  Deferred lanes queue their
        // point index and are re-projected exactly after the stream.
        // PF 5 (default): the same stream with contribute_lean's single-precision error terms and a contracted
        // transform, and the deferred lanes of the workgroup's four waves drained together (a wave defers ~0.4 %
        // of its points, a few per pass: one drain chunk per workgroup instead of one mostly idle chunk per wave).
        constexpr bool LEAN = PF == 5;
        const int nv = __builtin_amdgcn_readfirstlane(*npts);
        const int lane = tidx & 63;
        const int qcap = ((nv + stride - 1) / stride) * 64;
        int* q = dq + ((long)bidx * NW + (tidx >> 6)) * qcap;
        int qn = 0;
        auto acc = [&](const Proj& o, const float4 G, const float2 T) {
            if (LEAN) contribute_lean<METHOD>(A, W, errf, o, G, T, angle_res_inv, C);
            else contribute_fast<METHOD, 0>(A, W, o, G, T, 0, angle_res_inv, C);
        };
        const Gather gt{__builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(tg), 0, nRows * nCols * 16, 0x00020000),
                        __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(trg), 0, nRows * nCols * 8, 0x00020000)};
        const auto prs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(pts), 0, nv * 16, 0x00020000);
        struct Src { float4 p; bool valid; };
        auto ld = [&](int base) {        // out-of-range lanes read 0 (buffer bounds) and are not valid
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(prs, (base + lane) * 16, 0, 0);
            return Src{make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                                   __uint_as_float(v[3])), base + lane < nv};
        };
        auto prj = [&](const Src& x) {
            return project_fast<LEAN>(P, Lut3{x.p.x, x.p.y, x.p.z, x.valid}, x.p.w, nRows, nCols, angle_res_inv, asin_out);
        };
        auto defer = [&](Proj& o, int base) {
            const unsigned long long m = __ballot(o.fix);
            if (m) {
                const int pos = qn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                if (o.fix) { q[pos] = base + lane; o.vis = false; o.t = 0; }
                qn += __popcll(m);
            }
        };
        // XCD-aware stream order: workgroups are dispatched round-robin over the 8 XCDs, so with nb % 8 == 0
        // workgroup x runs on XCD x % 8; give each XCD one contiguous nb/8-workgroup slice of every stride
        // period, so a neighbourhood of the target's rows is gathered through one L2 instead of eight
        const int nbx = (int)gridDim.x;
        const int bx = (nbx & 7) ? (int)bidx : ((int)bidx & 7) * (nbx >> 3) + ((int)bidx >> 3);
        const int b0 = __builtin_amdgcn_readfirstlane((bx * TPB + (tidx & ~63)));
        if (b0 < nv) {
            const int n_it = (nv - 1 - b0) / stride + 1;
            auto base = [&](int k) { return b0 + (k < n_it ? k : n_it - 1) * stride; };
            Src sA = ld(base(0));
            Src sB = ld(base(1));
            Proj oA = prj(sA);
            defer(oA, base(0));
            float4 GA = gt.g(oA.t);
            float2 TA = gt.T(oA.t);
            for (int k = 0;; k += 2) {
                sA = ld(base(k + 2));
                Proj oB = prj(sB);
                if (k + 1 < n_it) defer(oB, base(k + 1));   // a clamped tail chunk is never accumulated
                const float4 GB = gt.g(oB.t);
                const float2 TB = gt.T(oB.t);
                acc(oA, GA, TA);
                if (k + 1 >= n_it) break;
                sB = ld(base(k + 3));
                oA = prj(sA);
                if (k + 2 < n_it) defer(oA, base(k + 2));
                GA = gt.g(oA.t);
                TA = gt.T(oA.t);
                acc(oB, GB, TB);
                if (k + 2 >= n_it) break;
            }
        }
        if (!LEAN && qn > 0) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            for (int s0 = 0; s0 < qn; s0 += 64) {
                const bool act = s0 + lane < qn;
                const int i = act ? q[s0 + lane] : 0;
                const float4 a = pts[i];
                Proj o = project_exact(P, Lut3{a.x, a.y, a.z, true}, a.w, nRows, nCols, half_nRows, angle_res_inv);
                o.vis = o.vis && act;
                o.t = o.vis ? o.t : 0;
                acc(o, gt.g(o.t), gt.T(o.t));
            }
        }
        if (LEAN) {
            // the workgroup's queues as one list (wave w's entries after those of waves < w), 64 entries per
            // drain chunk, chunk j on wave j % NW; the queue stores of other waves are ordered before the loads
            // by the workgroup-scope release / acquire of the barrier (one CU, one L1)
            if (lane == 0) s_qn[tidx >> 6] = qn;
            __syncthreads();
            int pre[NW + 1];
            pre[0] = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) pre[w + 1] = pre[w] + s_qn[w];
            const int tot = pre[NW];
            const int* qb = dq + (long)bidx * NW * qcap;
            for (int s0 = (tidx >> 6) * 64; s0 < tot; s0 += NW * 64) {
                const int g = s0 + lane;
                const bool act = g < tot;
                int w = 0;
#pragma unroll
                for (int v = 1; v < NW; ++v) w += g >= pre[v] ? 1 : 0;
                const int i = act ? qb[w * qcap + (g - pre[w])] : 0;
                const float4 a = pts[i];
                Proj o = project_exact(P, Lut3{a.x, a.y, a.z, true}, a.w, nRows, nCols, half_nRows, angle_res_inv);
                o.vis = o.vis && act;
                o.t = o.vis ? o.t : 0;
                acc(o, gt.g(o.t), gt.T(o.t));
            }
        }
    } else if (PF == 6 || PF == 10) {
        // (PF 10, experiment builds: the same body without the two-chunk software pipeline, at R360_PF10_MINB waves per
        // SIMD: latency hidden by more waves instead of a second chunk in flight)
        // Level 0 from the PACKED level-0 images (LevelBufs::pk, 4 B per pixel: range mm | luma << 16): the
        // source is streamed as the image itself, one wave = 64 consecutive pixels of one row (nCols % 64 == 0),
        // and the target {gray, depth} is gathered from the target's packed image (4 B instead of 8).  Per pass
        // and pair that reads 4 N + 20 V bytes instead of PF 5's 16 N_valid + 24 V, with the LUT point computed
        // from the row / column tables by the compaction's own float expressions (lut_point) and gray / depth by
        // the stitch's (luma * (float)(1/255), range * 0.001f): bit for bit the values PF 5 reads.  Pixels
        // without a valid depth ride along as invisible lanes (~10 % at level 0).  Projection, lean terms and the
        // workgroup drain as PF 5.
        const int npx = nRows * nCols;
        const int lane = tidx & 63;
        const int qcap = ((npx + stride - 1) / stride) * 64;
        int* q = dq + ((long)bidx * NW + (tidx >> 6)) * qcap;
        int qn = 0;
        const uint32_t* __restrict__ spk = J.spk;
        const auto rs_s = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(spk), 0, npx * 4, 0x00020000);
        const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(tg), 0, npx * 16, 0x00020000);
        const auto rs_t = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(J.tpk), 0, npx * 4, 0x00020000);
        auto gray_of = [](unsigned v) { return (float)(v >> 16) * (float)(1. / 255); };   // k_stitch4's expressions
        auto depth_of = [](unsigned v) { return (float)(v & 0xffffu) * 0.001f; };
#ifdef R360_EXP_NOGATHER   // experiment builds only (tools/exp_variants.sh): no target loads
        auto gG = [&](int t) { const float v = (float)(t & 1023) * 1e-3f; return make_float4(v, -v, v, 0.5f * v); };
        auto gT = [&](int t) { return (unsigned)(t & 0xffffff); };
#else
        auto gG = [&](int t) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs_g, t * 16, 0, 0);
            return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
        };
        auto gT = [&](int t) { return __builtin_amdgcn_raw_buffer_load_b32(rs_t, t * 4, 0, 0); };
#endif
#if R360_PK_ACC
        AccPk K;
        pk_zero(K);
#endif
        auto acc = [&](const Proj& o, const float4 G, unsigned tv) {
#ifdef R360_EXP_NOACC   // experiment builds only: keep the operands alive, skip the math
            A.h[0] += o.vis ? G.x + G.y + G.z + G.w + gray_of(tv) + depth_of(tv) + o.X + o.dist : 0.f;
            W.c28 += wave_count(o.vis);
            return;
#endif
#if R360_PK_ACC
            contribute_pk<METHOD>(K, W, errf, o, G, make_float2(gray_of(tv), depth_of(tv)), angle_res_inv, C);
#else
            contribute_lean<METHOD, false>(A, W, errf, o, G, make_float2(gray_of(tv), depth_of(tv)), angle_res_inv, C);
#endif
        };
        // row of a wave-uniform pixel index: a float estimate corrected by one step either way (exact for
        // pixel indices below 2^24, every level-0 size here)
        const float inv_cols = 1.f / (float)nCols;
        auto row_of = [&](int i) {
            int r = (int)((float)i * inv_cols);
            r -= (r * nCols > i) ? 1 : 0;
            r += ((r + 1) * nCols <= i) ? 1 : 0;
            return r;
        };
        struct Src { unsigned v; float sp, cp, st, ct; };
        int n_it_ = 0;
        // the source cursor: chunk k's first pixel, row and column, advanced by the stride in scalar registers
        // (SALU) and clamped at the last chunk, as base(k)
        int cur_k = 0, cur_i = 0, cur_r = 0, cur_c = 0;
        const int st_r = stride / nCols, st_c = stride - (stride / nCols) * nCols;
        // the column tables through buffer resources (32-bit offsets: one address VALU for both loads)
        const auto rs_st = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(sinth), 0, nCols * 4, 0x00020000);
        const auto rs_ct = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(costh), 0, nCols * 4, 0x00020000);
        auto ld = [&]() {
            const int co = (cur_c + lane) * 4;
            const Src x{__builtin_amdgcn_raw_buffer_load_b32(rs_s, (cur_i + lane) * 4, 0, 0), sinphi[cur_r],
                        cosphi[cur_r], __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_st, co, 0, 0)),
                        __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_ct, co, 0, 0))};
            if (cur_k + 1 < n_it_) {
                ++cur_k;
                cur_i += stride;
                cur_r += st_r;
                cur_c += st_c;
                if (cur_c >= nCols) { cur_c -= nCols; ++cur_r; }
            }
            return x;
        };
        auto prj = [&](const Src& x) {
            const float d = depth_of(x.v);
            return project_fast<true>(P, lut_point(d, x.sp, x.cp, x.st, x.ct, C), gray_of(x.v), nRows, nCols,
                                      angle_res_inv, asin_out);
        };
        auto defer = [&](Proj& o, int base) {
            const unsigned long long m = __ballot(o.fix);
            if (m) {
                const int pos = qn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                if (o.fix) { q[pos] = base + lane; o.vis = false; o.t = 0; }
                qn += __popcll(m);
            }
        };
        const int nbx = (int)gridDim.x;   // XCD-aware stream order (as PF 4 / 5)
        const int bx = (nbx & 7) ? (int)bidx : ((int)bidx & 7) * (nbx >> 3) + ((int)bidx >> 3);
        const int b0 = __builtin_amdgcn_readfirstlane((bx * TPB + (tidx & ~63)));
#ifdef R360_EXP_NOLOOP   // experiment builds only: the pass without its pixel loop (fixed costs)
        if (false) {
#else
        if (b0 < npx) {
#endif
            const int n_it = (npx - 1 - b0) / stride + 1;
            n_it_ = n_it;
            cur_i = b0;
            cur_r = __builtin_amdgcn_readfirstlane(row_of(b0));
            cur_c = b0 - cur_r * nCols;
            auto base = [&](int k) { return b0 + (k < n_it ? k : n_it - 1) * stride; };
            if constexpr (PF == 10) {
                for (int k = 0; k < n_it; ++k) {
                    const Src sx = ld();
                    Proj ox = prj(sx);
                    defer(ox, base(k));
                    const float4 Gx = gG(ox.t);
                    const unsigned Tx = gT(ox.t);
                    acc(ox, Gx, Tx);
                }
            } else {
            Src sA = ld();
            Src sB = ld();
            Proj oA = prj(sA);
            defer(oA, base(0));
            float4 GA = gG(oA.t);
            unsigned TA = gT(oA.t);
            for (int k = 0;; k += 2) {
                sA = ld();
                Proj oB = prj(sB);
                if (k + 1 < n_it) defer(oB, base(k + 1));   // a clamped tail chunk is never accumulated
                const float4 GB = gG(oB.t);
                const unsigned TB = gT(oB.t);
                acc(oA, GA, TA);
                if (k + 1 >= n_it) break;
                sB = ld();
                oA = prj(sA);
                if (k + 2 < n_it) defer(oA, base(k + 2));
                GA = gG(oA.t);
                TA = gT(oA.t);
                acc(oB, GB, TB);
                if (k + 2 >= n_it) break;
            }
            }
        }
        // the workgroup's deferred lanes, drained together (as PF 5)
        if (lane == 0) s_qn[tidx >> 6] = qn;
        __syncthreads();
        int pre[NW + 1];
        pre[0] = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) pre[w + 1] = pre[w] + s_qn[w];
        const int tot = pre[NW];
        const int* qb = dq + (long)bidx * NW * qcap;
        for (int s0 = (tidx >> 6) * 64; s0 < tot; s0 += NW * 64) {
            const int g = s0 + lane;
            const bool act = g < tot;
            int w = 0;
#pragma unroll
            for (int v = 1; v < NW; ++v) w += g >= pre[v] ? 1 : 0;
            const int i = act ? qb[w * qcap + (g - pre[w])] : 0;
            const unsigned v = spk[i];
            const int r = i / nCols, c = i - r * nCols;
            Proj o = project_exact(P, lut_point(depth_of(v), sinphi[r], cosphi[r], sinth[c], costh[c], C), gray_of(v),
                                   nRows, nCols, half_nRows, angle_res_inv);
            o.vis = o.vis && act;
            o.t = o.vis ? o.t : 0;
            acc(o, gG(o.t), gT(o.t));
        }
#if R360_PK_ACC
        pk_fold(A, K);
#endif
    } else if (PF == 8 || PF == 9) {
        // Coarse levels of batched launches from the level's {gray, depth} IMAGE instead of the source's compacted
        // points (round 6): frames that only enter batches then skip the per-frame source compaction (two launches per
        // frame).  PF 6's wave stream: one wave = 64 consecutive pixels, a cursor in scalar registers; where the rows
        // split into whole waves (cols % 64 == 0, PF 8) the row is wave-uniform (scalar sin / cos phi), otherwise (PF 9:
        // levels of 240 / 480 columns) a wave spans two rows and each lane takes its own (vector table loads).  The LUT point comes
        // from the tables by the compaction's float expressions (lut_point) and the target {gray, depth} is gathered as
        // a float2: per pixel the values, validity and lean terms of PF 5, summed in another lane order.
        const int npx = nRows * nCols;
        const int lane = tidx & 63;
        const int qcap = ((npx + stride - 1) / stride) * 64;
        int* q = dq + ((long)bidx * NW + (tidx >> 6)) * qcap;
        int qn = 0;
        constexpr bool whole = PF == 8;
        const auto rs_s = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(src), 0, npx * 8, 0x00020000);
        const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(tg), 0, npx * 16, 0x00020000);
        const auto rs_t = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(trg), 0, npx * 8, 0x00020000);
        const auto rs_sp = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(sinphi), 0, nRows * 4, 0x00020000);
        const auto rs_cp = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(cosphi), 0, nRows * 4, 0x00020000);
        const auto rs_st = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(sinth), 0, nCols * 4, 0x00020000);
        const auto rs_ct = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(costh), 0, nCols * 4, 0x00020000);
        auto f2 = [](decltype(__builtin_amdgcn_raw_buffer_load_b64(rs_s, 0, 0, 0)) v) {
            return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
        };
        auto gG = [&](int t) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs_g, t * 16, 0, 0);
            return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
        };
        auto gT = [&](int t) { return f2(__builtin_amdgcn_raw_buffer_load_b64(rs_t, t * 8, 0, 0)); };
        auto acc = [&](const Proj& o, const float4 G, const float2 T) {
            contribute_lean<METHOD>(A, W, errf, o, G, T, angle_res_inv, C);
        };
        const float inv_cols = 1.f / (float)nCols;
        auto row_of = [&](int i) {
            int r = (int)((float)i * inv_cols);
            r -= (r * nCols > i) ? 1 : 0;
            r += ((r + 1) * nCols <= i) ? 1 : 0;
            return r;
        };
        struct Src { float2 v; float sp, cp, st, ct; };
        int n_it_ = 0;
        int cur_k = 0, cur_i = 0, cur_r = 0, cur_c = 0;
        const int st_r = stride / nCols, st_c = stride - (stride / nCols) * nCols;
        auto ld = [&]() {
            int c = cur_c + lane, r = cur_r;
            float sp, cp;
            if constexpr (whole) {
                sp = sinphi[cur_r];
                cp = cosphi[cur_r];
            } else {   // the wave's pixels past the row end start the next row (nCols >= 64); past the image: depth 0
                const bool nx = c >= nCols;
                c -= nx ? nCols : 0;
                r += nx ? 1 : 0;
                sp = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_sp, r * 4, 0, 0));
                cp = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_cp, r * 4, 0, 0));
            }
            const Src x{f2(__builtin_amdgcn_raw_buffer_load_b64(rs_s, (cur_i + lane) * 8, 0, 0)), sp, cp,
                        __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_st, c * 4, 0, 0)),
                        __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_ct, c * 4, 0, 0))};
            if (cur_k + 1 < n_it_) {
                ++cur_k;
                cur_i += stride;
                cur_r += st_r;
                cur_c += st_c;
                if (cur_c >= nCols) { cur_c -= nCols; ++cur_r; }
            }
            return x;
        };
        auto prj = [&](const Src& x) {
            return project_fast<true>(P, lut_point(x.v.y, x.sp, x.cp, x.st, x.ct, C), x.v.x, nRows, nCols,
                                      angle_res_inv, asin_out);
        };
        auto defer = [&](Proj& o, int base) {
            const unsigned long long m = __ballot(o.fix);
            if (m) {
                const int pos = qn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                if (o.fix) { q[pos] = base + lane; o.vis = false; o.t = 0; }
                qn += __popcll(m);
            }
        };
        const int nbx = (int)gridDim.x;   // XCD-aware stream order (as PF 4 / 5 / 6)
        const int bx = (nbx & 7) ? (int)bidx : ((int)bidx & 7) * (nbx >> 3) + ((int)bidx >> 3);
        const int b0 = __builtin_amdgcn_readfirstlane((bx * TPB + (tidx & ~63)));
        if (b0 < npx) {
            const int n_it = (npx - 1 - b0) / stride + 1;
            n_it_ = n_it;
            cur_i = b0;
            cur_r = __builtin_amdgcn_readfirstlane(row_of(b0));
            cur_c = b0 - cur_r * nCols;
            auto base = [&](int k) { return b0 + (k < n_it ? k : n_it - 1) * stride; };
            Src sA = ld();
            Src sB = ld();
            Proj oA = prj(sA);
            defer(oA, base(0));
            float4 GA = gG(oA.t);
            float2 TA = gT(oA.t);
            for (int k = 0;; k += 2) {
                sA = ld();
                Proj oB = prj(sB);
                if (k + 1 < n_it) defer(oB, base(k + 1));   // a clamped tail chunk is never accumulated
                const float4 GB = gG(oB.t);
                const float2 TB = gT(oB.t);
                acc(oA, GA, TA);
                if (k + 1 >= n_it) break;
                sB = ld();
                oA = prj(sA);
                if (k + 2 < n_it) defer(oA, base(k + 2));
                GA = gG(oA.t);
                TA = gT(oA.t);
                acc(oB, GB, TB);
                if (k + 2 >= n_it) break;
            }
        }
        // the workgroup's deferred lanes, drained together (as PF 5)
        if (lane == 0) s_qn[tidx >> 6] = qn;
        __syncthreads();
        int pre[NW + 1];
        pre[0] = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) pre[w + 1] = pre[w] + s_qn[w];
        const int tot = pre[NW];
        const int* qb = dq + (long)bidx * NW * qcap;
        for (int s0 = (tidx >> 6) * 64; s0 < tot; s0 += NW * 64) {
            const int g = s0 + lane;
            const bool act = g < tot;
            int w = 0;
#pragma unroll
            for (int v = 1; v < NW; ++v) w += g >= pre[v] ? 1 : 0;
            const int i = act ? qb[w * qcap + (g - pre[w])] : 0;
            const float2 v = src[i];
            const int r = i / nCols, c = i - r * nCols;
            Proj o = project_exact(P, lut_point(v.y, sinphi[r], cosphi[r], sinth[c], costh[c], C), v.x, nRows, nCols,
                                   half_nRows, angle_res_inv);
            o.vis = o.vis && act;
            o.t = o.vis ? o.t : 0;
            acc(o, gG(o.t), gT(o.t));
        }
    } else if (PF == 7) {
        // PF 6 with a deeper software pipeline (sources two steps ahead of their projection, gathers two steps
        // ahead of their accumulation): the level-0 pass is bound by memory latency, not by VALU or bytes
        // Level 0 from the PACKED level-0 images (LevelBufs::pk, 4 B per pixel: range mm | luma << 16): the
        // source is streamed as the image itself, one wave = 64 consecutive pixels of one row (nCols % 64 == 0),
        // and the target {gray, depth} is gathered from the target's packed image (4 B instead of 8).  Per pass
        // and pair that reads 4 N + 20 V bytes instead of PF 5's 16 N_valid + 24 V, with the LUT point computed
        // from the row / column tables by the compaction's own float expressions (lut_point) and gray / depth by
        // the stitch's (luma * (float)(1/255), range * 0.001f): bit for bit the values PF 5 reads.  Pixels
        // without a valid depth ride along as invisible lanes (~10 % at level 0).  Projection, lean terms and the
        // workgroup drain as PF 5.
        const int npx = nRows * nCols;
        const int lane = tidx & 63;
        const int qcap = ((npx + stride - 1) / stride) * 64;
        int* q = dq + ((long)bidx * NW + (tidx >> 6)) * qcap;
        int qn = 0;
        const uint32_t* __restrict__ spk = J.spk;
        const auto rs_s = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(spk), 0, npx * 4, 0x00020000);
        const auto rs_g = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(tg), 0, npx * 16, 0x00020000);
        const auto rs_t = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(J.tpk), 0, npx * 4, 0x00020000);
        auto gray_of = [](unsigned v) { return (float)(v >> 16) * (float)(1. / 255); };   // k_stitch4's expressions
        auto depth_of = [](unsigned v) { return (float)(v & 0xffffu) * 0.001f; };
#ifdef R360_EXP_NOGATHER   // experiment builds only (tools/exp_variants.sh): no target loads
        auto gG = [&](int t) { const float v = (float)(t & 1023) * 1e-3f; return make_float4(v, -v, v, 0.5f * v); };
        auto gT = [&](int t) { return (unsigned)(t & 0xffffff); };
#else
        auto gG = [&](int t) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs_g, t * 16, 0, 0);
            return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
        };
        auto gT = [&](int t) { return __builtin_amdgcn_raw_buffer_load_b32(rs_t, t * 4, 0, 0); };
#endif
        auto acc = [&](const Proj& o, const float4 G, unsigned tv) {
#ifdef R360_EXP_NOACC   // experiment builds only: keep the operands alive, skip the math
            A.h[0] += o.vis ? G.x + G.y + G.z + G.w + gray_of(tv) + depth_of(tv) + o.X + o.dist : 0.f;
            W.c28 += wave_count(o.vis);
            return;
#endif
            contribute_lean<METHOD>(A, W, errf, o, G, make_float2(gray_of(tv), depth_of(tv)), angle_res_inv, C);
        };
        // row of a wave-uniform pixel index: a float estimate corrected by one step either way (exact for
        // pixel indices below 2^24, every level-0 size here)
        const float inv_cols = 1.f / (float)nCols;
        auto row_of = [&](int i) {
            int r = (int)((float)i * inv_cols);
            r -= (r * nCols > i) ? 1 : 0;
            r += ((r + 1) * nCols <= i) ? 1 : 0;
            return r;
        };
        struct Src { unsigned v; float sp, cp, st, ct; };
        auto ld = [&](int base) {                          // base: wave-uniform first pixel of a 64-pixel run
            const int r = __builtin_amdgcn_readfirstlane(row_of(base));
            const int c = base - r * nCols + lane;
            return Src{__builtin_amdgcn_raw_buffer_load_b32(rs_s, (base + lane) * 4, 0, 0), sinphi[r], cosphi[r],
                       sinth[c], costh[c]};
        };
        auto prj = [&](const Src& x) {
            const float d = depth_of(x.v);
            return project_fast<true>(P, lut_point(d, x.sp, x.cp, x.st, x.ct, C), gray_of(x.v), nRows, nCols,
                                      angle_res_inv, asin_out);
        };
        auto defer = [&](Proj& o, int base) {
            const unsigned long long m = __ballot(o.fix);
            if (m) {
                const int pos = qn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                if (o.fix) { q[pos] = base + lane; o.vis = false; o.t = 0; }
                qn += __popcll(m);
            }
        };
        const int nbx = (int)gridDim.x;   // XCD-aware stream order (as PF 4 / 5)
        const int bx = (nbx & 7) ? (int)bidx : ((int)bidx & 7) * (nbx >> 3) + ((int)bidx >> 3);
        const int b0 = __builtin_amdgcn_readfirstlane((bx * TPB + (tidx & ~63)));
        if (b0 < npx) {
            // three-step pipeline over chunk slots 0..2 (chunk h in slot h % 3, source slot (h + 1) % 3 refilled
            // with chunk h + 4): each step loads the source of chunk h + 4, projects chunk h + 2 (its source
            // loaded two steps earlier) and issues its gathers, and accumulates chunk h (gathered two steps
            // earlier).  A projected chunk keeps only its key {p', gray, target pixel}; |p'| and 1/|p'| are
            // recomputed by the same expressions when it is accumulated.
            const int n_it = (npx - 1 - b0) / stride + 1;
            auto base = [&](int k) { return b0 + (k < n_it ? k : n_it - 1) * stride; };
            struct Key { float X, Y, Z, g; int t; };   // t = target pixel, -1 when not visible
            auto stage_b = [&](const Src& x, int k, Key& K, float4& G, unsigned& T) {
                Proj o = prj(x);
                if (k < n_it) defer(o, base(k));   // a clamped tail chunk is never accumulated
                K = Key{o.X, o.Y, o.Z, o.gray_s, o.vis ? o.t : -1};
                G = gG(o.t);
                T = gT(o.t);
            };
            auto stage_c = [&](const Key& K, const float4 G, unsigned T) {
                Proj o;
                o.X = K.X; o.Y = K.Y; o.Z = K.Z; o.gray_s = K.g;
                const float d2 = K.X * K.X + K.Y * K.Y + K.Z * K.Z;   // project_fast's expressions
                o.dist_inv = __builtin_amdgcn_rsqf(d2);
                o.dist = r360m::sqrt_rn(d2);
                o.vis = K.t >= 0;
                o.t = o.vis ? K.t : 0;
                o.fix = false;
                acc(o, G, T);
            };
            Src S0 = ld(base(0)), S1 = ld(base(1)), S2 = ld(base(2));
            Key K0, K1, K2;
            float4 G0, G1, G2;
            unsigned T0, T1, T2;
            stage_b(S0, 0, K0, G0, T0);
            S0 = ld(base(3));
            stage_b(S1, 1, K1, G1, T1);
            for (int h = 0;; h += 3) {
                S1 = ld(base(h + 4));
                stage_b(S2, h + 2, K2, G2, T2);
                stage_c(K0, G0, T0);
                if (h + 1 >= n_it) break;
                S2 = ld(base(h + 5));
                stage_b(S0, h + 3, K0, G0, T0);
                stage_c(K1, G1, T1);
                if (h + 2 >= n_it) break;
                S0 = ld(base(h + 6));
                stage_b(S1, h + 4, K1, G1, T1);
                stage_c(K2, G2, T2);
                if (h + 3 >= n_it) break;
            }
        }
        // the workgroup's deferred lanes, drained together (as PF 5)
        if (lane == 0) s_qn[tidx >> 6] = qn;
        __syncthreads();
        int pre[NW + 1];
        pre[0] = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) pre[w + 1] = pre[w] + s_qn[w];
        const int tot = pre[NW];
        const int* qb = dq + (long)bidx * NW * qcap;
        for (int s0 = (tidx >> 6) * 64; s0 < tot; s0 += NW * 64) {
            const int g = s0 + lane;
            const bool act = g < tot;
            int w = 0;
#pragma unroll
            for (int v = 1; v < NW; ++v) w += g >= pre[v] ? 1 : 0;
            const int i = act ? qb[w * qcap + (g - pre[w])] : 0;
            const unsigned v = spk[i];
            const int r = i / nCols, c = i - r * nCols;
            Proj o = project_exact(P, lut_point(depth_of(v), sinphi[r], cosphi[r], sinth[c], costh[c], C), gray_of(v),
                                   nRows, nCols, half_nRows, angle_res_inv);
            o.vis = o.vis && act;
            o.t = o.vis ? o.t : 0;
            acc(o, gG(o.t), gT(o.t));
        }
    } else {
        // small levels: one pixel per thread, so the latency chain per thread is a quarter as long
        const int npx = nRows * nCols;
        for (int i = bidx * TPB + tidx; i < npx; i += stride) {
            const int r = i / nCols;
            const int c = i - r * nCols;
            const float2 a = src[i];
            one(a.y, a.x, sinphi[r], cosphi[r], sinth[c], costh[c], flag(i));
        }
    }
#ifdef R360_STAMPS
    const unsigned long long t_loop = __builtin_amdgcn_s_memrealtime();
    if (tidx == 0) {   // earliest block start / latest loop end over the grid
        if (bidx < 8192) {
            g_blk_stamps[0][bidx] = t_start;
            g_blk_stamps[1][bidx] = t_loop;
            unsigned hw, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            g_blk_stamps[2][bidx] = ((unsigned long long)xcc << 32) | hw;
        }
        // no grid-wide min / max here: 2 x 512 same-address atomics at the loop end serialised for ~10 us when
        // every workgroup finishes at once (coarse levels) and showed up as a ticket delay; the host takes
        // them from the per-workgroup stamps
    }
#endif

    // ---- stage 1: wave butterfly (f32) -> LDS -> per-workgroup fp64 record
    const int lane = tidx & 63, wid = tidx >> 6;
    if (PF >= 3 && lane == 0) { A.h[27] += (float)W.c27; A.h[28] += (float)W.c28; A.h[29] += (float)W.c29; }
    if (PF >= 5) A.err2 = (double)errf;
#ifdef R360_EXP_NOEPI   // experiment builds only
    if (A.h[0] == 1.2345f) S->dbg[7] = 1;
    return PASS_ARRIVED;
#endif
#ifdef R360_EXP_NOBFLY   // experiment builds only
    const float mine = A.h[lane & 31];
    const double e2 = A.err2, e2d = A.err2d;
#else
    const float mine = wave_reduce_scatter32(A.h, lane);
    const double e2 = wave_sum_d(A.err2);
    const double e2d = OCC ? wave_sum_d(A.err2d) : 0.0;
#endif
    if ((lane & 1) == 0) s_red[wid][scatter_slot(lane)] = mine;
    if (lane == 0) { s_err[wid] = e2; s_errd[wid] = e2d; }
    __syncthreads();
#ifdef R360_EXP_NOREC   // experiment builds only: no record, no ticket
    if (s_red[0][0] == 1.2345f) S->dbg[7] = 1;
    return PASS_ARRIVED;
#endif
    if (tidx < 32) {
        double v;
        if (tidx == R360_SUM_ERR2) {
            v = 0; for (int w = 0; w < NW; ++w) v += s_err[w];
        } else if (OCC && tidx == R360_SUM_ERR2D) {
            v = 0; for (int w = 0; w < NW; ++w) v += s_errd[w];
        } else {
            v = 0; for (int w = 0; w < NW; ++w) v += (double)s_red[w][tidx];
        }
        // write-through (sc1) store: visible at agent scope without an L2 write-back fence
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(partials) + (long)bidx * 32 + tidx,
                           (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
#if R360_POLL
#define R360_KPRE nullptr
    // ---- stage 2: record flags; the job's last workgroup polls them, reduces all records and runs the GN step
    // Every workgroup but the last stores this launch's sequence number (C.seq, unique per launch on the ctx)
    // into its own flag word once its record is drained (the sc1 record stores and the barrier as below); the
    // last workgroup of the job (dispatched after all the others, so it waits only on workgroups that have
    // started) reads the nb - 1 flags in parallel until every one holds C.seq.  No same-address
    // atomics: the arrival ticket serialised 512 simultaneous arrivals at the memory side (a coarse level's
    // workgroups all finish within a microsecond, and their ticket took ~12 us of the pass; profiles/r3_lone).
    {
        const int nb = (int)gridDim.x;
        if ((int)bidx != nb - 1) {
            if (tidx == 0)
                __hip_atomic_store(gcnt + bidx, C.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return PASS_ARRIVED;
        }
        for (int b = tidx; b < nb - 1; b += TPB)
            while (__hip_atomic_load(gcnt + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != C.seq)
                __builtin_amdgcn_s_sleep(1);
        __syncthreads();
    }
#else
    // ---- stage 2: arrival ticket; the last workgroup reduces all records and runs the GN step
    // Hand-off (MI355X_MICROARCH.md 'Valid forms', row 1): every record store is sc1 and drained by
    // its wave (vmcnt(0) above) before the barrier; one relaxed agent-scope add per workgroup; the
    // last adder reads every record with sc1 loads.  No buffer_wbl2 / buffer_inv fences: a release
    // fence per workgroup wrote back each XCD's dirty L2 (tens of us per pass).
    // Two-level ticket: agent-scope atomics on one address serialise at the memory side (~50 ns each,
    // 256 of them were ~13 us of every level-0 pass), so workgroups first count in 16 group counters
    // (4 KB apart) and only the last of each group takes the pass ticket: 32 + 16 deep instead of 512.
#if R360_GROUP_SUM
    // Two-level record sum along the two-level ticket: the last workgroup of ticket group g (records g, g + 16,
    // ...) sums its group's records into a group record (slot nb + g) while other groups are still arriving, and
    // the last group's workgroup then sums only the 16 group records.  Group sum: thread (s, q) adds records
    // j = s, s + 16 of the group (16 B of each, sc1 loads), then slot v is summed over s in order; the final sum
    // adds the group records in group order.  Fixed order for a given grid, so a job's sums are the same in any
    // batch; one load round on the last group's path instead of four (512 records, 8 in flight per lane).
    const int nb = (int)gridDim.x;
    const int ng = nb < R360_TICKET_GROUPS ? nb : R360_TICKET_GROUPS;
    if (tidx == 0) {
        const int g = (int)bidx % R360_TICKET_GROUPS;
        const unsigned gsz = (unsigned)((nb - g + R360_TICKET_GROUPS - 1) / R360_TICKET_GROUPS);
        const unsigned prev = __hip_atomic_fetch_add(gcnt + g * R360_TICKET_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == gsz - 1;
    }
    __syncthreads();
    if (!s_last) return PASS_ARRIVED;
    // The GN state, loaded by every group's last workgroup along with its group records: the step's workgroup then
    // has it in registers when it wins the pass ticket (the load after the ticket was ~1.2 us of every pass,
    // profiles/r4_gn).  Nothing writes the state during the pass but the ticket word, which the step resets.
    constexpr int NQ = (int)(sizeof(IcpState) / 16);
    static_assert(NQ <= TPB, "one 16-B word of the state per thread");
    uint4 st_q = {0u, 0u, 0u, 0u};
    if (!eval_only && (int)tidx < NQ) {   // sc1: a persistent launch's previous pass wrote it on another CU
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(__builtin_amdgcn_make_buffer_rsrc(S, 0, (int)sizeof(IcpState),
                                                                                               0x00020000),
                                                             (int)tidx * 16, 0, 16);
        st_q = make_uint4(v[0], v[1], v[2], v[3]);
    }
    unsigned long long kpre[4] = {0ull, 0ull, 0ull, 0ull};   // the span words pass_arrive updates
    if (tidx == 0) {
        const int lv = C.level & 7;
        kpre[0] = __hip_atomic_load(kt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        kpre[1] = __hip_atomic_load(kt + 1 + lv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        kpre[2] = __hip_atomic_load(kt + 9 + lv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        kpre[3] = __hip_atomic_load(kt + 18 + lv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#define R360_KPRE kpre
    {
        const int g = (int)bidx % R360_TICKET_GROUPS;
        const int gsz = (nb - g + R360_TICKET_GROUPS - 1) / R360_TICKET_GROUPS;
        const int q = tidx & 15, sj = tidx >> 4;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(partials, 0, (nb + R360_TICKET_GROUPS) * 256, 0x00020000);
        double a0 = 0.0, a1 = 0.0;
        for (int j = sj; j < gsz; j += 2 * RG) {
            const int j2 = j + RG < gsz ? j + RG : j;   // two loads in flight
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, ((g + j * R360_TICKET_GROUPS) * 16 + q) * 16, 0, 16);
            const auto y = __builtin_amdgcn_raw_buffer_load_b128(rs, ((g + j2 * R360_TICKET_GROUPS) * 16 + q) * 16, 0, 16);
            a0 += __longlong_as_double((long long)(((unsigned long long)x[1] << 32) | x[0]));
            a1 += __longlong_as_double((long long)(((unsigned long long)x[3] << 32) | x[2]));
            if (j2 != j) {
                a0 += __longlong_as_double((long long)(((unsigned long long)y[1] << 32) | y[0]));
                a1 += __longlong_as_double((long long)(((unsigned long long)y[3] << 32) | y[2]));
            }
        }
        s_fin[sj][2 * q] = a0;
        s_fin[sj][2 * q + 1] = a1;
        __syncthreads();
        if (tidx < 32) {
            double t = 0.0;
            for (int k = 0; k < RG; ++k) t += s_fin[k][tidx];
            __hip_atomic_store(reinterpret_cast<unsigned long long*>(partials) + (long)(nb + g) * 32 + tidx,
                               (unsigned long long)__double_as_longlong(t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    if (tidx == 0) {
        const unsigned p2 = __hip_atomic_fetch_add(&S->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = p2 == (unsigned)ng - 1;
    }
    __syncthreads();
    if (!s_last) return PASS_ARRIVED;
    if (tidx < R360_TICKET_GROUPS)   // every group is complete: reset its counter for the next pass
        __hip_atomic_store(gcnt + tidx * R360_TICKET_STRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
#define R360_KPRE nullptr
    if (tidx == 0) {
        const int nb = (int)gridDim.x;
        const int ng = nb < R360_TICKET_GROUPS ? nb : R360_TICKET_GROUPS;
        const int g = (int)bidx % R360_TICKET_GROUPS;
        const unsigned gsz = (unsigned)((nb - g + R360_TICKET_GROUPS - 1) / R360_TICKET_GROUPS);
        const unsigned prev = __hip_atomic_fetch_add(gcnt + g * R360_TICKET_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int last = 0;
        if (prev == gsz - 1) {
            const unsigned p2 = __hip_atomic_fetch_add(&S->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = (p2 == (unsigned)ng - 1);
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return PASS_ARRIVED;
    if (tidx < R360_TICKET_GROUPS)   // every group is complete: reset its counter for the next pass
        __hip_atomic_store(gcnt + tidx * R360_TICKET_STRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
#endif
#ifdef R360_STAMPS
    const unsigned long long t_ticket = __builtin_amdgcn_s_memrealtime();
#endif
#if !R360_POLL && R360_GROUP_SUM
    if (tidx < 16 * R360_TICKET_GROUPS) {   // the group records, 16 B per lane
        const int q = tidx & 15, g = tidx >> 4;
        double a0 = 0.0, a1 = 0.0;
        if (g < ng) {
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(partials, 0, (nb + R360_TICKET_GROUPS) * 256, 0x00020000);
            const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, ((nb + g) * 16 + q) * 16, 0, 16);
            a0 = __longlong_as_double((long long)(((unsigned long long)x[1] << 32) | x[0]));
            a1 = __longlong_as_double((long long)(((unsigned long long)x[3] << 32) | x[2]));
        }
        s_fin[g][2 * q] = a0;
        s_fin[g][2 * q + 1] = a1;
    }
#else
    {
        // fixed-order reduction of the per-workgroup records: lane q of a 16-lane group loads bytes
        // 16q..16q+15 of records g, g+RG, ... with L1-bypassing (sc1) 16-B buffer loads, 8 in flight;
        // then thread v sums slot v over the groups in order
        const int q = tidx & 15, g = tidx >> 4;
        const int nb = (int)gridDim.x;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(partials, 0, nb * 256, 0x00020000);
        double a0 = 0.0, a1 = 0.0;
        auto add = [&](const decltype(__builtin_amdgcn_raw_buffer_load_b128(rs, 0, 0, 16))& x) {
            a0 += __longlong_as_double((long long)(((unsigned long long)x[1] << 32) | x[0]));
            a1 += __longlong_as_double((long long)(((unsigned long long)x[3] << 32) | x[2]));
        };
        int r = g;
        for (; r + 7 * RG < nb; r += 8 * RG) {
            decltype(__builtin_amdgcn_raw_buffer_load_b128(rs, 0, 0, 16)) x[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) x[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((r + j * RG) * 16 + q) * 16, 0, 16);
#pragma unroll
            for (int j = 0; j < 8; ++j) add(x[j]);
        }
        for (; r < nb; r += RG) add(__builtin_amdgcn_raw_buffer_load_b128(rs, (r * 16 + q) * 16, 0, 16));
        s_fin[g][2 * q] = a0;
        s_fin[g][2 * q + 1] = a1;
    }
#endif
    __syncthreads();
    if (tidx < 32) {
        double t = 0.0;
        for (int g = 0; g < RG; ++g) t += s_fin[g][tidx];
        s_fin[0][tidx] = t;
    }
    __syncthreads();
#ifdef R360_STAMPS
    const unsigned long long t_recs = __builtin_amdgcn_s_memrealtime();
#endif
    if (eval_only) {
        if (tidx < 32) S->sums[tidx] = s_fin[0][tidx];
#ifdef R360_STAMPS
        if (tidx == 0) {
            const unsigned long long mn = __hip_atomic_load(&S->dbg[8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long mx = __hip_atomic_load(&S->dbg[9], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            S->dbg[5] = mn; S->dbg[6] = mx; S->dbg[8] = ~0ull; S->dbg[9] = 0;
            S->dbg[0] = t_start; S->dbg[1] = t_loop; S->dbg[2] = t_ticket; S->dbg[3] = t_recs;
            S->dbg[4] = __builtin_amdgcn_s_memrealtime();
        }
#endif
        if (tidx == 0) {
            S->ticket = 0;
            pass_arrive(kt, true, C.level, R360_KPRE);   // the job's last workgroup
        }
        return PASS_STEPPED;
    }
    // Stage the whole state in LDS with one coalesced 16-B access per thread, run the step on the LDS copy (one
    // lane walking global memory serialises ~150 dependent accesses, ~35 us), then write it back the same way.
    uint4* sq = reinterpret_cast<uint4*>(&s_state);
#if !R360_POLL && R360_GROUP_SUM
    if ((int)tidx < NQ) sq[tidx] = st_q;   // loaded with the group records
#else
    constexpr int NQ = (int)(sizeof(IcpState) / 16);
    for (int q = tidx; q < NQ; q += TPB) sq[q] = reinterpret_cast<const uint4*>(S)[q];
#endif
    __syncthreads();
    gn_step_block(&s_state, s_fin[0], C, first, &s_gn, tidx);
    if (tidx == 0) {
        s_state.ticket = 0;
#ifdef R360_STAMPS
        s_state.dbg[5] = s_state.dbg[8]; s_state.dbg[6] = s_state.dbg[9];
        s_state.dbg[8] = ~0ull; s_state.dbg[9] = 0;
#endif
    }
    __syncthreads();
    if constexpr (PERSIST) {
        // write-through (sc1) stores, drained by every wave before the barrier the hand-off follows; the last
        // 16 B (the fault word that a timed-out waiter may set) are not written
        const auto rsS = __builtin_amdgcn_make_buffer_rsrc(S, 0, (int)sizeof(IcpState), 0x00020000);
        for (int q = tidx; q < NQ - 1; q += TPB) {
            const uint4 v = sq[q];
            const u32x4 w = {v.x, v.y, v.z, v.w};
            __builtin_amdgcn_raw_buffer_store_b128(w, rsS, q * 16, 0, 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        for (int q = tidx; q < NQ; q += TPB) reinterpret_cast<uint4*>(S)[q] = sq[q];
    }
#ifdef R360_STAMPS
    if (tidx == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long st[5] = {t_start, t_loop, t_ticket, t_recs, __builtin_amdgcn_s_memrealtime()};
        for (int k = 0; k < 5; ++k) __hip_atomic_store(&S->dbg[k], st[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#endif
    if constexpr (PERSIST) __syncthreads();   // every wave's state stores drained before the span and the hand-off
    if (tidx == 0) {   // the job's last workgroup
        if (PERSIST && gridDim.y > 1)   // a batched persistent level launch: its span is closed by the last exit
            __hip_atomic_fetch_add(kt + 18 + (C.level & 7), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            pass_arrive(kt, true, C.level, R360_KPRE, PERSIST);
    }
#undef R360_KPRE
    return PASS_STEPPED;
}

// PF 9 (coarse levels whose rows do not split into whole waves: per-lane rows, one more table pair live) at 4 waves per
// SIMD: at 5 its pipelined chunks spilled 20 B per lane; the levels it serves are the two smallest
template <int METHOD, int PF, int TOP, int OCC>
#ifndef R360_PF10_MINB
#define R360_PF10_MINB 6
#endif
__global__ __launch_bounds__(TPB, PF == 9 ? 4 : PF == 10 ? R360_PF10_MINB : R360_ICP_MINB) void k_icp_pass(const IcpJobs jobs, const float* __restrict__ sinphi,
                                                 const float* __restrict__ cosphi, const float* __restrict__ sinth,
                                                 const float* __restrict__ costh, int nRows, int nCols,
                                                 IcpConst C, int first, int eval_only,
                                                 unsigned long long* __restrict__ kt,
                                                 const uint8_t* __restrict__ occf) {
    (void)icp_pass_body<METHOD, PF, TOP, OCC, false>(jobs, sinphi, cosphi, sinth, costh, nRows, nCols, C, first,
                                                     eval_only, kt, occf, (int)threadIdx.x, (int)blockIdx.x);
}

// ---- persistent level launch (lone alignments, plain pass: PF 6 at level 0, PF 5 above)
// The level's 1 + maxIters passes in ONE launch on the pass grid of k_icp_pass (same workgroups, same pixel
// order, same records: the sums and poses are bit for bit those of the per-pass launches).  Between passes the
// step's workgroup publishes the pass generation (base + k + 1) after its state and span stores have drained;
// every other workgroup's lane 0 polls it (sc1 loads, s_sleep) and the workgroup joins at a barrier, then
// reads the new state with sc1 loads.  A level that converged ends the loop in every workgroup at once (they
// all read the same published state), so no launch is dispatched for its remaining passes (a stopped pass was
// a full-grid dispatch whose workgroups exit at entry, 29 of a lone pair's 65 launches), and the ~3 us kernel
// boundary of every pass becomes a one-flag hand-off.  base: the generation word at the launch start (every
// workgroup reads it before its first arrival, and nothing is published before all have arrived).  Every wait
// is bounded (R360_PERSIST_SPIN_TICKS): a timed-out waiter sets S->fault and leaves, and so do the others at
// their next wait, so the grid always drains.  The host launches it only when the grid fits one resident round
// with a workgroup per CU to spare (icp_level_persist_grid) and no other persistent launch of the process is in
// flight.
#ifndef R360_PERSIST_SLEEP
#define R360_PERSIST_SLEEP 2   // s_sleep between polls (units of 64 clocks)
#endif
#ifndef R360_PERSIST_SPIN_TICKS
#define R360_PERSIST_SPIN_TICKS 50000000ull   // 0.5 s of the 100 MHz s_memrealtime clock
#endif
#if R360_POLL || defined(R360_EXP_NOEPI) || defined(R360_EXP_NOREC)
#define R360_PERSIST_BUILT 0   // these experiment bodies have no step workgroup
#else
#define R360_PERSIST_BUILT 1
#endif
#ifndef R360_LEVEL_PF0
#define R360_LEVEL_PF0 6   // the level-0 form of the persistent launch (experiment variant lpf7: PF 7's deeper pipeline)
#endif
#ifndef R360_LEVEL_MINB
#define R360_LEVEL_MINB 3   // waves per SIMD: a lone pass puts 2 workgroups on a CU, so registers are free up to 3
#endif
// The level loop of a persistent launch, for job blockIdx.y (its own state, records, tickets and generation word).
template <int METHOD, int PF, int TOP>
__device__ __forceinline__ void icp_level_loop(const IcpJobs& jobs, const float* __restrict__ sinphi,
                                               const float* __restrict__ cosphi, const float* __restrict__ sinth,
                                               const float* __restrict__ costh, int nRows, int nCols, const IcpConst& C,
                                               int passes, unsigned long long* __restrict__ kt) {
    __shared__ int s_go;
    IcpState* S = jobs.j[blockIdx.y].S;
    unsigned* gen = jobs.j[blockIdx.y].gcnt + R360_PERSIST_FLAG_WORD;
    unsigned base = 0;
    if (threadIdx.x == 0) base = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int k = 0; k < passes; ++k) {
        // the pass's operands laundered per iteration (empty asm): otherwise the compiler hoists the body's
        // loop-invariant address and table arithmetic out of the pass loop, and the values it keeps live across
        // the whole pass spilled to scratch (288 B per lane) and were reloaded inside the pixel loop
        int tid = (int)threadIdx.x, bid = (int)blockIdx.x, nr = nRows, nc = nCols;
        const float *sp = sinphi, *cp = cosphi, *st = sinth, *ct = costh;
        unsigned long long* ktl = kt;
        asm volatile("" : "+v"(tid));
        asm volatile("" : "+s"(bid), "+s"(nr), "+s"(nc));
        asm volatile("" : "+s"(sp), "+s"(cp), "+s"(st), "+s"(ct), "+s"(ktl));
        const int r = icp_pass_body<METHOD, PF, TOP, 0, true>(jobs, sp, cp, st, ct, nr, nc, C, k == 0 ? 1 : 0, 0, ktl,
                                                              nullptr, tid, bid);
        if (r == PASS_SKIPPED || k + 1 == passes) break;   // stopped (uniform), or the level's last pass
        if (threadIdx.x == 0) {
            const unsigned tag = base + (unsigned)k + 1u;
            int go = 1;
            if (r == PASS_STEPPED) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(gen, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tag) {
                    __builtin_amdgcn_s_sleep(R360_PERSIST_SLEEP);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > R360_PERSIST_SPIN_TICKS) { go = 0; break; }
                }
                if (!go) __hip_atomic_store(&S->fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            s_go = go;
        }
        __syncthreads();
        if (!s_go) break;
    }
}

template <int METHOD, int PF, int TOP>
__global__ __launch_bounds__(TPB, R360_LEVEL_MINB) void k_icp_level(const IcpJobs jobs, const float* __restrict__ sinphi,
                                                  const float* __restrict__ cosphi, const float* __restrict__ sinth,
                                                  const float* __restrict__ costh, int nRows, int nCols,
                                                  IcpConst C, int passes, unsigned long long* __restrict__ kt) {
    icp_level_loop<METHOD, PF, TOP>(jobs, sinphi, cosphi, sinth, costh, nRows, nCols, C, passes, kt);
}

// ---- batched persistent coarse levels (round 6, experiment builds: measured slower, see launch_icp_levels_batch): ONE
// launch runs a coarse level of every job of a batch, each job on
// its own R360_COARSE_WG workgroups looping over the level's 1 + maxIters passes with the hand-off above (per-job
// generation word; a job that stops leaves the loop, so no launch is spent on converged passes).  Per batch that
// replaces 4 x 11 per-pass launches (most exiting at entry once their jobs converged, each with its launch gap on the
// dense stream, profiles/r6_s8) with 4.  A job's workgroups never wait on another job's, so the launch needs no
// resident round: workgroups are dispatched in index order (x, then the job y), the earliest unfinished job's
// workgroups are dispatched before any later job's, and each job's <= R360_COARSE_WG workgroups fit the GPU.  The
// bounded waits of the hand-off stay as the guard (a timed-out job faults, its batch returns an error).  The last
// workgroup to exit closes the launch's in-kernel span.  3 waves per SIMD: inside the level loop the pass keeps more
// values live (158 VGPRs; at 4 / 5 waves it spilled 52 / 148 B per lane).
#if R360_EXPERIMENTS
template <int METHOD, int PF>
__global__ __launch_bounds__(TPB, 3) void k_icp_levels_batch(
        const IcpJobs jobs, const float* __restrict__ sinphi, const float* __restrict__ cosphi,
        const float* __restrict__ sinth, const float* __restrict__ costh, int nRows, int nCols, IcpConst C, int passes,
        unsigned long long* __restrict__ kt) {
    icp_level_loop<METHOD, PF, 0>(jobs, sinphi, cosphi, sinth, costh, nRows, nCols, C, passes, kt);
    if (threadIdx.x == 0) {
        const unsigned long long total = (unsigned long long)gridDim.x * gridDim.y;
        const unsigned long long prev = __hip_atomic_fetch_add(kt + 17, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == total - 1) {
            __hip_atomic_store(kt + 17, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int lv = C.level & 7;
            const unsigned long long t0 = __hip_atomic_load(kt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            __hip_atomic_fetch_add(kt + 1 + lv, t1 > t0 ? t1 - t0 : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(kt + 9 + lv, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}
#endif

// ---------------------------------------------------------------- occlusion variants (§8(f)1)
// Per pass, before the fused pass and at the same pose:
//   k_occ_project  per source pixel: target pixel (the fused pass's exact decision), 1/|p'| with the
//                  reference's IEEE division, the Occ2 depth-outlier filter; counts per target pixel
//   k_occ_scan*    exclusive scan of the counts (per-target list offsets)
//   k_occ_scatter  source indices grouped by target pixel (counts return to zero)
//   k_occ_resolve  per target pixel, in LUT (source index) order: the Z-buffer's accepted points
//                  (prefix maxima of 1/|p'|), the last accepted one, and the last point
constexpr int OCC_SCAN_TPB = 1024, OCC_SCAN_V = 4, OCC_SCAN_ITEMS = OCC_SCAN_TPB * OCC_SCAN_V;

__device__ __forceinline__ bool pass_skipped(const IcpState* S, int first, int eval_only) {
    return S->stop || (!first && !S->active && !eval_only);
}

__device__ __forceinline__ Pose12 pass_pose(const IcpState* S, int first, int eval_only) {
    const float* pm = (first && !eval_only) ? S->pose : S->cand;
    Pose12 P;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) P.R[r * 3 + c] = pm[c * 4 + r];
        P.t[r] = pm[12 + r];
    }
    return P;
}

template <int OCC>
__global__ void __launch_bounds__(256) k_occ_project(const float2* __restrict__ src, const float2* __restrict__ trg,
                                                    const float* __restrict__ sinphi, const float* __restrict__ cosphi,
                                                    const float* __restrict__ sinth, const float* __restrict__ costh,
                                                    int nRows, int nCols, IcpConst C, const IcpState* S, int first,
                                                    int eval_only, int* __restrict__ tgt, float* __restrict__ dinv,
                                                    uint8_t* __restrict__ flags, int* __restrict__ cnt) {
    if (pass_skipped(S, first, eval_only)) return;
    const Pose12 P = pass_pose(S, first, eval_only);
    const float angle_res = (float)(2 * R360_PI / nCols);
    const float angle_res_inv = 1 / angle_res;
    const float half_nRows = (float)(0.5 * nRows - 0.5);
    const int npx = nRows * nCols;
    const int stride = gridDim.x * blockDim.x;
    // wave-uniform trip count (project_fix votes across the wave)
    for (int i0 = blockIdx.x * blockDim.x + (threadIdx.x & ~63); i0 < npx; i0 += stride) {
        const int i = min(i0 + (int)(threadIdx.x & 63), npx - 1);
        const bool own = i0 + (int)(threadIdx.x & 63) < npx;
        const int r = i / nCols, c = i - (i / nCols) * nCols;
        const float2 a = src[i];
        Proj o = project(P, a.y, a.x, sinphi[r], cosphi[r], sinth[c], costh[c], nRows, nCols, half_nRows,
                         angle_res_inv, C);
        project_fix(o, nRows, nCols, half_nRows, angle_res_inv);
        if (!own) continue;
        int t = -1;
        float di = 0.f;
        if (o.vis) {
            di = 1.f / o.dist;                                  // the reference's dist_inv (IEEE)
            bool keep = true;
            if (OCC == 2) keep = !(fabsf(trg[o.t].y - o.dist) > 0.3f);   // thresDepthOutliers (:4525, :3790)
            if (keep) {
                t = o.t;
                atomicAdd(cnt + t, 1);
            }
        }
        tgt[i] = t;
        dinv[i] = di;
        flags[i] = 0;
    }
}

// exclusive scan of cnt[0..n) into off[0..n] in three steps (workgroup scans, scan of the workgroup
// totals, add); off[n] = total
__device__ int occ_block_exscan(int v, int* sh, int& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    __syncthreads();
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int k = 0; k < nw; ++k) { const int t = sh[k]; sh[k] = acc; acc += t; }
        sh[nw] = acc;
    }
    __syncthreads();
    total = sh[nw];
    return sh[wid] + x - v;
}

__global__ void __launch_bounds__(OCC_SCAN_TPB) k_occ_scan1(const int* __restrict__ cnt, int n, int* __restrict__ off,
                                                          int* __restrict__ bsum, const IcpState* S, int first,
                                                          int eval_only) {
    __shared__ int sh[17];
    if (pass_skipped(S, first, eval_only)) return;
    const int j = blockIdx.x * OCC_SCAN_ITEMS + threadIdx.x * OCC_SCAN_V;
    int v[OCC_SCAN_V], t = 0;
#pragma unroll
    for (int k = 0; k < OCC_SCAN_V; ++k) { v[k] = j + k < n ? cnt[j + k] : 0; t += v[k]; }
    int tot;
    int e = occ_block_exscan(t, sh, tot);
#pragma unroll
    for (int k = 0; k < OCC_SCAN_V; ++k)
        if (j + k < n) { off[j + k] = e; e += v[k]; }
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(OCC_SCAN_TPB) k_occ_scan2(int* __restrict__ bsum, int nb, int* __restrict__ off,
                                                          int n, const IcpState* S, int first, int eval_only) {
    __shared__ int sh[17];
    if (pass_skipped(S, first, eval_only)) return;
    int acc = 0;
    for (int b0 = 0; b0 < nb; b0 += OCC_SCAN_TPB) {
        const int b = b0 + threadIdx.x;
        const int v = b < nb ? bsum[b] : 0;
        int tot;
        const int e = occ_block_exscan(v, sh, tot);
        if (b < nb) bsum[b] = acc + e;
        acc += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) off[n] = acc;
}

__global__ void __launch_bounds__(OCC_SCAN_TPB) k_occ_scan3(const int* __restrict__ bsum, int n, int* __restrict__ off,
                                                          const IcpState* S, int first, int eval_only) {
    if (pass_skipped(S, first, eval_only)) return;
    const int j = blockIdx.x * OCC_SCAN_ITEMS + threadIdx.x * OCC_SCAN_V;
    const int add = bsum[blockIdx.x];
#pragma unroll
    for (int k = 0; k < OCC_SCAN_V; ++k)
        if (j + k < n) off[j + k] += add;
}

__global__ void k_occ_scatter(const int* __restrict__ tgt, int n, const int* __restrict__ off, int* __restrict__ cnt,
                              int* __restrict__ list, const IcpState* S, int first, int eval_only) {
    if (pass_skipped(S, first, eval_only)) return;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int t = tgt[i];
        if (t < 0) continue;
        const int pos = atomicSub(cnt + t, 1) - 1;
        list[off[t] + pos] = i;
    }
}

__global__ void k_occ_resolve(const int* __restrict__ off, int n, const int* __restrict__ list,
                              const float* __restrict__ dinv, uint8_t* __restrict__ flags, const IcpState* S,
                              int first, int eval_only) {
    if (pass_skipped(S, first, eval_only)) return;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const int b = off[t], m = off[t + 1] - b;
        if (m == 0) continue;
        if (m == 1) { flags[list[b]] = OCC_ACC | OCC_OWN | OCC_WIN; continue; }
        // m points hit this target pixel: walk them in source-index order.  invDepthBuffer starts at 0
        // and keeps the last accepted 1/|p'|, so a point is accepted iff 1/|p'| >= every earlier one
        int prev = -1, last_acc = -1;
        float zmax = 0.f;
        for (int k = 0; k < m; ++k) {
            int nxt = 0x7fffffff;                           // smallest source index above prev
            for (int q = 0; q < m; ++q) {
                const int i = list[b + q];
                if (i > prev && i < nxt) nxt = i;
            }
            prev = nxt;
            const float d = dinv[nxt];
            const bool acc = !(zmax > 0.f && d < zmax);
            if (acc) { zmax = d; last_acc = nxt; }
            flags[nxt] = acc ? OCC_ACC : 0;
        }
        flags[last_acc] |= OCC_OWN;
        flags[prev] |= OCC_WIN;                             // prev = largest source index
    }
}

}  // namespace

namespace {
__global__ void k_libm(const float* x, const float* y, const float* z, int n, float* as, float* at) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { as[i] = r360m::asinf(x[i]); at[i] = r360m::atan2f_sel(y[i], z[i]); }
}
}  // namespace

// Test hook: evaluates the asinf/atan2f port on the host or on the device.
extern "C" int r360_libm_eval(const float* x, const float* y, const float* z, int n, float* asin_out,
                              float* atan2_out, int on_device) {
    if (!on_device) {
        for (int i = 0; i < n; ++i) { asin_out[i] = r360m::asinf(x[i]); atan2_out[i] = r360m::atan2f_sel(y[i], z[i]); }
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
    int b = (units + TPB - 1) / TPB;  // one 4-pixel unit per thread up to the cap
    if (b > 1024) b = 1024;
    return b < 1 ? 1 : b;
}

namespace {
// Test hook: the PF 3 pass's decision for LUT points (lx, ly, lz) at pose P — the fast projection, or
// the exact one for a flagged (deferred) lane — against the exact program alone: pixel-decision
// mismatches (must be 0; the PF 5 form with the contracted transform is checked on the same points) and
// deferrals.
__global__ void k_proj_check(const float* __restrict__ X, const float* __restrict__ Y, const float* __restrict__ Z,
                             int n, Pose12 P, int nRows, int nCols, unsigned long long* __restrict__ out) {
    const float angle_res = (float)(2 * R360_PI / nCols);
    const float angle_res_inv = 1 / angle_res;
    const float half_nRows = (float)(0.5 * nRows - 0.5);
    unsigned long long mism = 0, fb = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        Lut3 l;
        l.x = X[i]; l.y = Y[i]; l.z = Z[i]; l.valid = true;
        const Proj e = project_exact(P, l, 0.f, nRows, nCols, half_nRows, angle_res_inv);
        Proj f = project_fast(P, l, 0.f, nRows, nCols, angle_res_inv, asin_out_for(nRows, nCols));
        Proj fl = project_fast<true>(P, l, 0.f, nRows, nCols, angle_res_inv, asin_out_for(nRows, nCols));  // PF 5
        if (f.fix) { f = e; ++fb; }
        if (fl.fix) fl = e;
        const bool same = f.vis == e.vis && f.t == e.t && fl.vis == e.vis && fl.t == e.t;
        mism += same ? 0 : 1;
        if (!same) { out[2] = (unsigned long long)i; out[3] = (unsigned long long)f.t; out[4] = (unsigned long long)e.t; }
    }
    atomicAdd(out, mism);
    atomicAdd(out + 1, fb);
}

int proj_check(const float* X, const float* Y, const float* Z, int n, const float* pose, int nRows, int nCols,
               unsigned long long* mismatches, unsigned long long* fallbacks) {
    Pose12 P;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) P.R[r * 3 + c] = pose ? pose[c * 4 + r] : (r == c ? 1.f : 0.f);
        P.t[r] = pose ? pose[12 + r] : 0.f;
    }
    float *dx, *dy, *dz;
    unsigned long long* dout;
    R360_HIP(hipMalloc(&dx, sizeof(float) * n));
    R360_HIP(hipMalloc(&dy, sizeof(float) * n));
    R360_HIP(hipMalloc(&dz, sizeof(float) * n));
    R360_HIP(hipMalloc(&dout, 64));
    R360_HIP(hipMemcpy(dx, X, sizeof(float) * n, hipMemcpyHostToDevice));
    R360_HIP(hipMemcpy(dy, Y, sizeof(float) * n, hipMemcpyHostToDevice));
    R360_HIP(hipMemcpy(dz, Z, sizeof(float) * n, hipMemcpyHostToDevice));
    R360_HIP(hipMemset(dout, 0, 64));
    hipLaunchKernelGGL(k_proj_check, dim3(1024), dim3(256), 0, 0, dx, dy, dz, n, P, nRows, nCols, dout);
    R360_HIP(hipGetLastError());
    unsigned long long h[8];
    R360_HIP(hipMemcpy(h, dout, 64, hipMemcpyDeviceToHost));
    if (h[0] && R360_KNOB_STR("R360_PROJ_DEBUG"))
        fprintf(stderr, "proj mismatch at %llu: fast pixel %lld exact pixel %lld\n", h[2], (long long)h[3], (long long)h[4]);
    (void)hipFree(dx); (void)hipFree(dy); (void)hipFree(dz); (void)hipFree(dout);
    *mismatches = h[0];
    *fallbacks = h[1];
    return 0;
}

}  // namespace

namespace {
// Test hook: sqrt_rn / div_rn against the compiler's IEEE sqrtf and '/' on hashed operands spanning the
// ranges the pass feeds them (squared ranges 1e-4..1e4, weights and residuals 1e-5..1e3).
__device__ __forceinline__ float hash_unit(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return (float)(x >> 8) * (1.f / 16777216.f);
}
__global__ void k_rn_check(unsigned n, unsigned seed, unsigned long long* __restrict__ out) {
    unsigned long long ms = 0, md = 0;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const unsigned k = i * 3u + seed * 0x9e3779b9u;
        const float x = exp2f(hash_unit(k) * 26.6f - 13.3f);            // 1e-4 .. 1e4
        const float a = exp2f(hash_unit(k + 1) * 26.6f - 16.6f);        // 1e-5 .. 1e3
        const float b = exp2f(hash_unit(k + 2) * 26.6f - 16.6f);
        volatile float xs = x, as = a, bs = b;
        ms += __float_as_uint(r360m::sqrt_rn(x)) != __float_as_uint(sqrtf(xs));
        md += __float_as_uint(r360m::div_rn(a, b)) != __float_as_uint(as / bs);
    }
    atomicAdd(out, ms);
    atomicAdd(out + 1, md);
}
}  // namespace

namespace {
// the row form (the GN step's) and the wave form (pinhole / robot steps) must agree: -1 where they do not
__global__ void k_rank6(const float* __restrict__ M, int n, int* __restrict__ out) {
    const int m = blockIdx.x, lane = threadIdx.x;
    if (m >= n) return;
    const float a = lane < 36 ? M[m * 36 + lane] : 0.f;
    const int rw = wave_rank6(a, lane);
    float r[6];
    const int i = lane < 6 ? lane : 0;
#pragma unroll
    for (int j = 0; j < 6; ++j) r[j] = M[m * 36 + i * 6 + j];
    const int rr = rank6_rows(r, lane);
    if (lane == 0) out[m] = rr == rw ? rr : -1;
}

// x = -H^-1 g by the GN step's row-per-lane solve (solve6_rows_dpp); one wave per system
__global__ void k_solve6(const double* __restrict__ H, const double* __restrict__ g, int n, double* __restrict__ x) {
    const int m = blockIdx.x, lane = threadIdx.x;
    if (m >= n) return;
    const int i = lane < 6 ? lane : 0;
    double a[7], xs[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) a[j] = H[m * 36 + i * 6 + j];
    a[6] = -g[m * 6 + i];
    solve6_rows_dpp(a, lane, xs);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 6; ++k) x[m * 6 + k] = xs[k];
}
}  // namespace

// Test hook: the GN step's solve (icp_la.inc solve6_rows_dpp) on n systems (H row-major n x 36, g n x 6) -> x n x 6.
extern "C" int r360_solve6(const double* H, const double* g, int n, double* x) {
    if (!H || !g || !x || n <= 0) { r360_set_error("r360_solve6: bad arguments"); return -2; }
    double *dH, *dg, *dx;
    R360_HIP(hipMalloc(&dH, sizeof(double) * 36 * (size_t)n));
    R360_HIP(hipMalloc(&dg, sizeof(double) * 6 * (size_t)n));
    R360_HIP(hipMalloc(&dx, sizeof(double) * 6 * (size_t)n));
    R360_HIP(hipMemcpy(dH, H, sizeof(double) * 36 * (size_t)n, hipMemcpyHostToDevice));
    R360_HIP(hipMemcpy(dg, g, sizeof(double) * 6 * (size_t)n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_solve6, dim3(n), dim3(64), 0, 0, dH, dg, n, dx);
    R360_HIP(hipGetLastError());
    R360_HIP(hipMemcpy(x, dx, sizeof(double) * 6 * (size_t)n, hipMemcpyDeviceToHost));
    (void)hipFree(dH); (void)hipFree(dg); (void)hipFree(dx);
    return 0;
}

// Test hook: the device rank test (wave_rank6, the ILL-POSED check of alignFrames360 :4682 / alignFrames
// :4345 / RegisterDensePhotoICP :443) on n row-major 6x6 float matrices.
extern "C" int r360_rank6(const float* M, int n, int* ranks) {
    if (!M || !ranks || n <= 0) { r360_set_error("r360_rank6: bad arguments"); return -2; }
    float* dM;
    int* dr;
    R360_HIP(hipMalloc(&dM, sizeof(float) * 36 * (size_t)n));
    R360_HIP(hipMalloc(&dr, sizeof(int) * (size_t)n));
    R360_HIP(hipMemcpy(dM, M, sizeof(float) * 36 * (size_t)n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_rank6, dim3(n), dim3(64), 0, 0, dM, n, dr);
    R360_HIP(hipGetLastError());
    R360_HIP(hipMemcpy(ranks, dr, sizeof(int) * (size_t)n, hipMemcpyDeviceToHost));
    (void)hipFree(dM); (void)hipFree(dr);
    return 0;
}

extern "C" int r360_rn_check(unsigned n, unsigned seed, unsigned long long out[2]) {
    unsigned long long* d;
    R360_HIP(hipMalloc(&d, 16));
    R360_HIP(hipMemset(d, 0, 16));
    hipLaunchKernelGGL(k_rn_check, dim3(1024), dim3(256), 0, 0, n, seed, d);
    R360_HIP(hipGetLastError());
    R360_HIP(hipMemcpy(out, d, 16, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return 0;
}

extern "C" int r360_proj_check(const float* X, const float* Y, const float* Z, int n, int nRows, int nCols,
                               unsigned long long* mismatches, unsigned long long* fallbacks) {
    return proj_check(X, Y, Z, n, nullptr, nRows, nCols, mismatches, fallbacks);
}

extern "C" int r360_proj_check_pose(const float* lx, const float* ly, const float* lz, int n, const float pose[16],
                                    int nRows, int nCols, unsigned long long* mismatches,
                                    unsigned long long* fallbacks) {
    return proj_check(lx, ly, lz, n, pose, nRows, nCols, mismatches, fallbacks);
}

#ifdef R360_STAMPS
// Diagnostic build only: per-workgroup start / loop-end stamps and hardware ids of the last pass (out: 3 x 8192).
extern "C" int r360_debug_block_stamps(unsigned long long* out, int n) {
    if (n > 8192) n = 8192;
    R360_HIP(hipDeviceSynchronize());
    R360_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_blk_stamps), sizeof(unsigned long long) * 8192 * 3));
    return n;
}
#endif

// The pass forms the product library holds (each covered by the parity suite): PF 6 at level 0 (TOP = 1) of batched
// launches, PF 5 on the other levels and at level 0 of lone alignments (and where the packed image is not streamable), PF 3 / PF 0 for the occlusion
// variants (PF 0 where rows do not split into whole waves).  PF 1 / 2 / 4 / 7 and the forced-form knobs exist only
// in the experiment builds (R360_EXPERIMENTS, make exp).
template <int M, int PF>
static int launch_pass(r360_ctx* ctx, int nb, int njobs, const IcpJobs& jobs, const LevelBufs& Ls,
                        const LevelTrig& T, const IcpConst& C, int first, int eval_only, bool top) {
    void (*kern)(const IcpJobs, const float*, const float*, const float*, const float*, int, int, IcpConst, int, int,
                 unsigned long long*, const uint8_t*) = nullptr;
    if (C.occ) {
        // PF 4 / 5 / 6 (compacted or packed source) have no occlusion form: the occlusion flags are per source pixel
        constexpr int PFO = PF >= 4 ? 3 : PF;
        if constexpr (PFO == 0 || PFO == 3 || R360_EXPERIMENTS)
            kern = C.occ == 1 ? k_icp_pass<M, PFO, 0, 1> : k_icp_pass<M, PFO, 0, 2>;
    } else if constexpr (PF == 5 || R360_EXPERIMENTS) {
        kern = top ? k_icp_pass<M, PF, 1, 0> : k_icp_pass<M, PF, 0, 0>;
    } else if constexpr (PF == 6) {
        kern = k_icp_pass<M, PF, 1, 0>;   // level 0 only
    } else if constexpr (PF == 8 || PF == 9) {
        kern = k_icp_pass<M, PF, 0, 0>;   // the coarse levels of batched launches
    }
    if (!kern) {
        r360_set_error("k_icp_pass: form PF %d (occlusion %d, top %d) is not in this build", PF, C.occ, (int)top);
        return -1;
    }
    hipLaunchKernelGGL(kern, dim3(nb, njobs), dim3(TPB), 0, ctx->stream, jobs, T.sinphi, T.cosphi, T.sinth,
                       T.costh, Ls.rows, Ls.cols, C, first, eval_only, ctx->d_ktime, ctx->occ_flags);
    return 0;
}

int ensure_defer(r360_ctx* ctx, long n_pixels) {
    // per wave ceil(npx / stride) * 64 entries over nb * NW waves: <= npx + nb * TPB for any nb
    const long need = n_pixels + (long)ctx->partials_cap * TPB;
    if (ctx->defer_cap >= need) return 0;
    R360_HIP(hipSetDevice(ctx->device));
    R360_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->d_defer) R360_HIP(hipFree(ctx->d_defer));
    ctx->d_defer = nullptr;
    ctx->defer_cap = 0;
    R360_HIP(hipMalloc(&ctx->d_defer, sizeof(int) * need));
    ctx->defer_cap = need;
    return 0;
}

// Sizes the batch buffers of ctx for n jobs over frames of up to n_pixels level-0 pixels (synchronises the
// ctx stream when they grow).  Job j: state j, partials_cap records, its own ticket groups and queue.
int ensure_batch(r360_ctx* ctx, int n, long n_pixels) {
    const long dneed = n_pixels + (long)ctx->partials_cap * TPB;
    if (ctx->batch_cap >= n && ctx->bdefer_cap >= dneed) return 0;
    const int cap = n > ctx->batch_cap ? n : ctx->batch_cap;
    const long dcap = dneed > ctx->bdefer_cap ? dneed : ctx->bdefer_cap;
    R360_HIP(hipSetDevice(ctx->device));
    R360_HIP(hipStreamSynchronize(ctx->stream));
    (void)hipFree(ctx->d_bstate); (void)hipFree(ctx->d_bpartials); (void)hipFree(ctx->d_bgticket);
    (void)hipFree(ctx->d_bdefer); (void)hipHostFree(ctx->h_bstate);
    ctx->d_bstate = nullptr; ctx->d_bpartials = nullptr; ctx->d_bgticket = nullptr; ctx->d_bdefer = nullptr;
    ctx->h_bstate = nullptr;
    ctx->batch_cap = 0; ctx->bdefer_cap = 0;
    const size_t tk = (size_t)R360_TICKET_GROUPS * R360_TICKET_STRIDE;
    R360_HIP(hipMalloc(&ctx->d_bstate, sizeof(IcpState) * cap));
    R360_HIP(hipMalloc(&ctx->d_bpartials, sizeof(double) * 32 * (size_t)ctx->partials_cap * cap));
    R360_HIP(hipMalloc(&ctx->d_bgticket, sizeof(unsigned) * tk * cap));
    // zeroed on the ctx stream, ahead of the batch's passes: hipMemset (null stream) neither orders with the
    // non-blocking ctx stream nor completes before returning, and recycled memory left the first batches' group
    // counters non-zero now and then (a wrong last workgroup: one pair in a few hundred off the single-pair result)
    R360_HIP(hipMemsetAsync(ctx->d_bgticket, 0, sizeof(unsigned) * tk * cap, ctx->stream));
    R360_HIP(hipMalloc(&ctx->d_bdefer, sizeof(int) * (size_t)dcap * cap));
    R360_HIP(hipHostMalloc(&ctx->h_bstate, sizeof(IcpState) * cap, hipHostMallocDefault));
    ctx->batch_cap = cap;
    ctx->bdefer_cap = dcap;
    return 0;
}

// grid of one job's pass at level `level` of `geom` (the same for every job of a batch): the pass form and
// the number of workgroups
struct PassGrid { int pf, nb; };
static PassGrid pass_grid(const r360_ctx* ctx, const LevelBufs& Ls, int occ, int njobs = 1, bool batched = false,
                          bool pts = false) {
    // 4-pixel units on the large levels, one pixel per thread where that still fits one resident
    // round (latency-bound small levels); R360_ICP_PF=0/1 forces one form (experiments)
    static const int pf_env = R360_KNOB("R360_ICP_PF", -1);
    static const int cap_env = R360_KNOB("R360_ICP_CAP", -1);
    // one resident round: CUs x workgroups per CU of the launched form (grid-stride beyond it)
    static const int cus = [] {   // thread-safe one-time query (contexts may be driven from several threads)
        int dev = 0, n = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n;
    }();
    const int npx = Ls.rows * Ls.cols;
    // PF 4 (compacted source points) for the plain pass; the occlusion variants index their flags by source
    // pixel and keep the image stream (PF 3 where rows split into whole waves)
    // level 0 (the only level with a packed image) streams the packed images where rows split into whole waves, in
    // batched launches: PF 6 reads 0.64x PF 5's bytes with fewer instructions, which a full chip of waves turns into
    // throughput.  A lone alignment's pass (two workgroups per CU, latency-bound) runs PF 5 over the source's
    // compacted level-0 points (pts: built with the frame, r360_frame::compact_all): only valid pixels, no deferred
    // lanes, the shorter dependent chain; level-0 pass 26.9 -> 24.2 us in-kernel, lone pair 0.92 -> 0.85 ms
    // (profiles/r5_lone).  The two forms sum the same pixels in different orders (equal to rounding).
    // Round 6: the coarse levels of batched launches stream the level's image too (PF 8, levels of >= 64 columns), so
    // the frames of batched alignments need no compacted source points at all (the sequence runner's ring frames skip
    // the two compaction launches per frame).  A lone alignment keeps PF 5 where its source has the level's points
    // (pts), and streams the image where it has not.
    const bool pk_ok = Ls.pk != nullptr && Ls.cols % 64 == 0;
    static const bool coarse_pf5 = R360_KNOB("R360_COARSE_PF5", 0) != 0;   // experiment builds: round 5's coarse form
    const bool img_ok = !pk_ok && Ls.cols >= 64 && !coarse_pf5;
    const int pf_img = pk_ok ? 6 : img_ok ? (Ls.cols % 64 == 0 ? 8 : 9) : 5;
    const int pf_dflt = occ ? ((Ls.cols % 64 == 0) ? 3 : 0) : (batched || !pts ? pf_img : 5);
    const bool env_ok = pf_env >= 0 && !(pf_env >= 4 && occ) && !((pf_env == 6 || pf_env == 7 || pf_env == 10) && !pk_ok) &&
                        !(pf_env == 8 && Ls.cols % 64 != 0) && !(pf_env == 9 && Ls.cols < 64);
    const int pf = R360_EXPERIMENTS && env_ok ? pf_env : pf_dflt;
    // workgroups per job and pass: 2 per CU (one resident round holds occ_q.per[pf] per CU; a batched launch
    // fills the rest with other jobs, and fewer records per job shorten the reduction tail)
    // workgroups per job and pass: a fixed number per level size, never a function of the batch, so that a
    // pair's sums (pixels to waves, records in workgroup order) and thus its pose are the same in any batch
    // and on any number of ranks.  R360_ICP_WG_TOTAL (experiment only: breaks that) splits a per-launch total
    // over the launch's jobs.
    // Batched launches (r360_align360_batch_*, the dense queue): one workgroup per CU and job, so a wave streams twice
    // the chunks of a lone pass and the per-workgroup tail (the exact re-projection of the deferred lanes, the record
    // reduction) is paid over twice the pixels: 1535 -> 1588-1595 pairs/s, dense alone 2205 -> 2274 (profiles/r5_cap).
    // A lone alignment keeps two per CU: with the GPU to itself it is latency-bound, and one per CU made a lone pair
    // 0.94 -> 1.16 ms.  Every batch of any size (and every rank) uses the batched grid, so a pair's batched result is
    // the same in any batch; a lone alignment sums the same pixels over twice the records (within rounding of it).
    static const int cap_batch_env = R360_KNOB("R360_ICP_CAP_BATCH", -1);
    int cap = cap_env > 0 ? cap_env : 2 * cus;
    if (batched) cap = cap_batch_env > 0 ? cap_batch_env : cus;
    static const int tot_env = R360_KNOB("R360_ICP_WG_TOTAL", -1);
    if (tot_env > 0) cap = ((tot_env / (njobs > 0 ? njobs : 1) + 7) / 8) * 8;
    if (cap > ctx->partials_cap - R360_TICKET_GROUPS) cap = ctx->partials_cap - R360_TICKET_GROUPS;   // + group records
    // at least R360_ICP_PXT points per thread (default 1; 8 measured no faster): the coarse levels (a quarter, ... of
    // level 0) then run on a few hundred / dozen workgroups per pair instead of one thread per point, which
    // shortens their record / ticket / final-sum tail (level 0 at VGA has ~19 per thread on the capped grid)
    static const int pxt_env = R360_KNOB("R360_ICP_PXT", -1);
    // Batched launches take at least 8 points per thread (round 5): levels 2-4 then run on 75 / 19 / 5 workgroups per
    // job instead of 256 / 150 / 38 (level 0 and 1 stay at the one-per-CU cap), so a batch's coarse passes need fewer
    // CU slots (under the pipelines' load their first workgroups waited for slots, profiles/r5_trace) and sum fewer
    // records: +0.9 % in an A/B (profiles/r5_envab/pxt/, r5_prep2/pxt8/).  The grid still depends only on the level size.
    const int pxt = pxt_env > 0 ? pxt_env : (batched ? 8 : 1);
    int nb = pf == 1 ? icp_blocks_for(npx) : (npx + TPB * pxt - 1) / (TPB * pxt);
    if (nb > cap) nb = cap;
    if (nb < 1) nb = 1;
    return {pf, nb};
}

// deferred-queue entries one job's PF 3 / PF 4 pass needs: per wave ceil(npx / stride) * 64
static long defer_need(int npx, int nb) {
    const long stride = (long)nb * TPB;
    return (long)nb * (TPB / 64) * (((npx + stride - 1) / stride) * 64);
}

static int launch_jobs(r360_ctx* ctx, const IcpJobs& jobs, int njobs, const LevelBufs& Ls, const LevelTrig& T,
                       int level, int method, const IcpConst& C0, int first, int eval_only, const PassGrid& G) {
    IcpConst C = C0;
    if (++ctx->icp_seq == 0) ++ctx->icp_seq;   // the record flags start (and may stale) at 0
    C.seq = ctx->icp_seq;
    const char* name = level == 0 ? "k_icp_pass_L0" : "k_icp_pass";
    const int slot = timing_begin(ctx, name);
    const int pf = G.pf, nb = G.nb;
    const bool top = level == 0;
#if R360_EXPERIMENTS
#define R360_LAUNCH_EXP(M)                                                                               \
        else if (pf == 1) rc = launch_pass<M, 1>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top); \
        else if (pf == 2) rc = launch_pass<M, 2>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top); \
        else if (pf == 4) rc = launch_pass<M, 4>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top); \
        else if (pf == 7) rc = launch_pass<M, 7>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top); \
        else if (pf == 10) rc = launch_pass<M, 10>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top);
#else
#define R360_LAUNCH_EXP(M)
#endif
#define R360_LAUNCH(M)                                                                                   \
    do {                                                                                                 \
        if (pf == 3) rc = launch_pass<M, 3>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top);      \
        else if (pf == 5) rc = launch_pass<M, 5>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top); \
        else if (pf == 6) rc = launch_pass<M, 6>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top); \
        else if (pf == 8) rc = launch_pass<M, 8>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top); \
        else if (pf == 9) rc = launch_pass<M, 9>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top); \
        R360_LAUNCH_EXP(M)                                                                               \
        else rc = launch_pass<M, 0>(ctx, nb, njobs, jobs, Ls, T, C, first, eval_only, top);              \
    } while (0)
    int rc = 0;
    if (method == R360_PHOTO_CONSISTENCY) R360_LAUNCH(R360_PHOTO_CONSISTENCY);
    else if (method == R360_DEPTH_CONSISTENCY) R360_LAUNCH(R360_DEPTH_CONSISTENCY);
    else R360_LAUNCH(R360_PHOTO_DEPTH);
#undef R360_LAUNCH
#undef R360_LAUNCH_EXP
    timing_end(ctx, slot);
    if (rc) return rc;
    R360_HIP(hipGetLastError());
    return 0;
}

int launch_icp_jobs(r360_ctx* ctx, const IcpJobs& jobs, int n, const r360_frame* geom, int level, int method,
                    const IcpConst& C, int first, int eval_only) {
    if (C.occ) { r360_set_error("batched passes: occlusion variants run one alignment per launch"); return -2; }
    if (n < 1 || n > R360_MAX_BATCH) { r360_set_error("batched passes: %d jobs (1..%d)", n, R360_MAX_BATCH); return -2; }
    const LevelBufs& Ls = geom->lv[level];
    const PassGrid G = pass_grid(ctx, Ls, 0, n, true);
    if (G.pf >= 3 && ctx->bdefer_cap < defer_need(Ls.rows * Ls.cols, G.nb)) {
        r360_set_error("batched passes: deferred-pixel queues not sized for %d pixels", Ls.rows * Ls.cols);
        return -1;
    }
    return launch_jobs(ctx, jobs, n, Ls, geom->calib->trig[level], level, method, C, first, eval_only, G);
}

// ---- batched persistent coarse levels (k_icp_levels_batch, experiment builds only: R360_COARSE_PERSIST=1): at most
// R360_COARSE_WG workgroups per job, PF 8 / 9.  Measured slower than the per-pass launches in the pipelined bench (1690.7 /
// 1696.4 vs 1738.0 / 1739.0 pairs/s alternating, profiles/r6_s9): the levels' workgroups, resident at 3 waves per SIMD
// and spinning between passes, hold CU slots the pipelines' frame and plane kernels wait for.  Returns 1 (launch the
// level pass by pass) in the product library and whenever the level has no persistent batched form.
int launch_icp_levels_batch(r360_ctx* ctx, const IcpJobs& jobs, int n, const r360_frame* geom, int level, int method,
                            const IcpConst& C0, int passes) {
#if !R360_EXPERIMENTS
    (void)ctx; (void)jobs; (void)n; (void)geom; (void)level; (void)method; (void)C0; (void)passes;
    return 1;
#else
    // R360_COARSE_WG: workgroups per job (1: no hand-off waits at all); R360_COARSE_MIN_LEVEL: the finest level run
    // this way (the finer ones pass by pass)
    static const int coarse_wg = R360_KNOB("R360_COARSE_WG", 64);
    static const int coarse_min = R360_KNOB("R360_COARSE_MIN_LEVEL", 1);
    static const bool persist = R360_KNOB("R360_COARSE_PERSIST", 0) != 0;
    if (level == 0 || level < coarse_min || C0.occ || !persist || !R360_PERSIST_BUILT) return 1;
    if (n < 1 || n > R360_MAX_BATCH) { r360_set_error("batched passes: %d jobs (1..%d)", n, R360_MAX_BATCH); return -2; }
    const LevelBufs& Ls = geom->lv[level];
    PassGrid G = pass_grid(ctx, Ls, 0, n, true);
    if (G.pf != 8 && G.pf != 9) return 1;
    if (G.nb > coarse_wg) G.nb = coarse_wg;
    if (ctx->bdefer_cap < defer_need(Ls.rows * Ls.cols, G.nb)) {
        r360_set_error("batched passes: deferred-pixel queues not sized for %d pixels", Ls.rows * Ls.cols);
        return -1;
    }
    const LevelTrig& T = geom->calib->trig[level];
    IcpConst C = C0;
    if (++ctx->icp_seq == 0) ++ctx->icp_seq;
    C.seq = ctx->icp_seq;
    void (*kern)(const IcpJobs, const float*, const float*, const float*, const float*, int, int, IcpConst, int,
                 unsigned long long*) = nullptr;
    auto pick = [&](auto m) {
        constexpr int M = decltype(m)::value;
        kern = G.pf == 8 ? k_icp_levels_batch<M, 8> : k_icp_levels_batch<M, 9>;
    };
    if (method == R360_PHOTO_CONSISTENCY) pick(std::integral_constant<int, R360_PHOTO_CONSISTENCY>{});
    else if (method == R360_DEPTH_CONSISTENCY) pick(std::integral_constant<int, R360_DEPTH_CONSISTENCY>{});
    else pick(std::integral_constant<int, R360_PHOTO_DEPTH>{});
    const int slot = timing_begin(ctx, "k_icp_levels");
    hipLaunchKernelGGL(kern, dim3(G.nb, n), dim3(TPB), 0, ctx->stream, jobs, T.sinphi, T.cosphi, T.sinth, T.costh,
                       Ls.rows, Ls.cols, C, passes, ctx->d_ktime);
    timing_end(ctx, slot);
    R360_HIP(hipGetLastError());
    return 0;
#endif
}

// ---- persistent level launch (k_icp_level): resident-round check and launch
template <int M, int PF, int TOP>
static int level_blocks_per_cu() {   // the occupancy query for the instantiation (one device model per process)
    static const int n = [] {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_icp_level<M, PF, TOP>, TPB, 0) != hipSuccess) b = 0;
        return b;
    }();
    return n;
}

static int level_blocks_per_cu(int method, int pf) {
    auto by = [&](auto m) {
        constexpr int M = decltype(m)::value;
        return pf == 6 ? level_blocks_per_cu<M, R360_LEVEL_PF0, 1>() : level_blocks_per_cu<M, 5, 0>();
    };
    if (method == R360_PHOTO_CONSISTENCY) return by(std::integral_constant<int, R360_PHOTO_CONSISTENCY>{});
    if (method == R360_DEPTH_CONSISTENCY) return by(std::integral_constant<int, R360_DEPTH_CONSISTENCY>{});
    return by(std::integral_constant<int, R360_PHOTO_DEPTH>{});
}

bool icp_level_persist_ok(r360_ctx* ctx, const r360_frame* src, int level, int method) {
    if (!R360_PERSIST_BUILT) return false;
    const LevelBufs& Ls = src->lv[level];
    const PassGrid G = pass_grid(ctx, Ls, 0, 1, false, (src->compacted >> level) & 1u);
    if (G.pf != 5 && G.pf != 6) return false;   // the product forms of the plain pass
    if (G.pf >= 3 && ctx->defer_cap < defer_need(Ls.rows * Ls.cols, G.nb)) return false;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return false;
    // the occupancy answer can be one workgroup per CU high (MI355X_MICROARCH.md, residency): keep one spare
    const int per_cu = level_blocks_per_cu(method, G.pf);
    return per_cu >= 2 && G.nb <= (per_cu - 1) * cus;
}

int launch_icp_level_persist(r360_ctx* ctx, const r360_frame* trg, const r360_frame* src, int level, int method,
                             const IcpConst& C0, int passes) {
    const LevelBufs& Ls = src->lv[level];
    const LevelBufs& Lt = trg->lv[level];
    const LevelTrig& T = src->calib->trig[level];
    const PassGrid G = pass_grid(ctx, Ls, 0, 1, false, (src->compacted >> level) & 1u);
    if (C0.occ || (G.pf != 5 && G.pf != 6) || !R360_PERSIST_BUILT) {
        r360_set_error("persistent level launch: plain pass forms only");
        return -1;
    }
    IcpJobs jobs;
    IcpJob& J = jobs.j[0];
    J.src = Ls.p0; J.trg = Lt.p0; J.tg = Lt.tg; J.pts = Ls.pts; J.npts = src->d_npts + level;
    J.spk = Ls.pk; J.tpk = Lt.pk;
    J.S = ctx->d_state; J.partials = ctx->d_partials; J.gcnt = ctx->d_gticket; J.dq = ctx->d_defer;
    IcpConst C = C0;
    if (++ctx->icp_seq == 0) ++ctx->icp_seq;
    C.seq = ctx->icp_seq;
    const int slot = timing_begin(ctx, level == 0 ? "k_icp_level_L0" : "k_icp_level");
    void (*kern)(const IcpJobs, const float*, const float*, const float*, const float*, int, int, IcpConst, int,
                 unsigned long long*) = nullptr;
    auto pick = [&](auto m) {
        constexpr int M = decltype(m)::value;
        kern = G.pf == 6 ? k_icp_level<M, R360_LEVEL_PF0, 1> : k_icp_level<M, 5, 0>;
    };
    if (method == R360_PHOTO_CONSISTENCY) pick(std::integral_constant<int, R360_PHOTO_CONSISTENCY>{});
    else if (method == R360_DEPTH_CONSISTENCY) pick(std::integral_constant<int, R360_DEPTH_CONSISTENCY>{});
    else pick(std::integral_constant<int, R360_PHOTO_DEPTH>{});
    hipLaunchKernelGGL(kern, dim3(G.nb, 1), dim3(TPB), 0, ctx->stream, jobs, T.sinphi, T.cosphi, T.sinth, T.costh,
                       Ls.rows, Ls.cols, C, passes, ctx->d_ktime);
    timing_end(ctx, slot);
    R360_HIP(hipGetLastError());
    return 0;
}

int launch_icp_level(r360_ctx* ctx, const r360_frame* trg, const r360_frame* src, int level, int method,
                     const IcpConst& C, int first, int eval_only) {
    const LevelBufs& Ls = src->lv[level];
    const LevelBufs& Lt = trg->lv[level];
    const LevelTrig& T = src->calib->trig[level];
    const PassGrid G = pass_grid(ctx, Ls, C.occ, 1, false, (src->compacted >> level) & 1u);
    const int npx = Ls.rows * Ls.cols;
    if (G.pf >= 3 && ctx->defer_cap < defer_need(npx, G.nb)) {   // one queue per wave, room for every pixel
        r360_set_error("deferred-pixel queue not sized for %d pixels (ensure_defer)", npx);
        return -1;
    }
    if (C.occ) {   // occlusion flags of this pass's pose (same stream, before the fused pass)
        if (ctx->occ_cap < npx) {
            (void)hipFree(ctx->occ_tgt); (void)hipFree(ctx->occ_dinv); (void)hipFree(ctx->occ_flags);
            (void)hipFree(ctx->occ_cnt); (void)hipFree(ctx->occ_off); (void)hipFree(ctx->occ_list);
            (void)hipFree(ctx->occ_bsum);
            const long n = npx;
            R360_HIP(hipMalloc(&ctx->occ_tgt, sizeof(int) * n));
            R360_HIP(hipMalloc(&ctx->occ_dinv, sizeof(float) * n));
            R360_HIP(hipMalloc(&ctx->occ_flags, n));
            R360_HIP(hipMalloc(&ctx->occ_cnt, sizeof(int) * n));
            R360_HIP(hipMalloc(&ctx->occ_off, sizeof(int) * (n + 1)));
            R360_HIP(hipMalloc(&ctx->occ_list, sizeof(int) * n));
            R360_HIP(hipMalloc(&ctx->occ_bsum, sizeof(int) * (n / OCC_SCAN_ITEMS + 2)));
            R360_HIP(hipMemsetAsync(ctx->occ_cnt, 0, sizeof(int) * n, ctx->stream));
            ctx->occ_cap = n;
        }
        const int b256 = (npx + 255) / 256, bscan = (npx + OCC_SCAN_ITEMS - 1) / OCC_SCAN_ITEMS;
        const int slot = timing_begin(ctx, "k_occ");
        hipStream_t st = ctx->stream;
        if (C.occ == 1)
            hipLaunchKernelGGL(k_occ_project<1>, dim3(b256), dim3(256), 0, st, Ls.p0, Lt.p0, T.sinphi, T.cosphi,
                               T.sinth, T.costh, Ls.rows, Ls.cols, C, ctx->d_state, first, eval_only, ctx->occ_tgt,
                               ctx->occ_dinv, ctx->occ_flags, ctx->occ_cnt);
        else
            hipLaunchKernelGGL(k_occ_project<2>, dim3(b256), dim3(256), 0, st, Ls.p0, Lt.p0, T.sinphi, T.cosphi,
                               T.sinth, T.costh, Ls.rows, Ls.cols, C, ctx->d_state, first, eval_only, ctx->occ_tgt,
                               ctx->occ_dinv, ctx->occ_flags, ctx->occ_cnt);
        hipLaunchKernelGGL(k_occ_scan1, dim3(bscan), dim3(OCC_SCAN_TPB), 0, st, ctx->occ_cnt, npx, ctx->occ_off,
                           ctx->occ_bsum, ctx->d_state, first, eval_only);
        hipLaunchKernelGGL(k_occ_scan2, dim3(1), dim3(OCC_SCAN_TPB), 0, st, ctx->occ_bsum, bscan, ctx->occ_off, npx,
                           ctx->d_state, first, eval_only);
        hipLaunchKernelGGL(k_occ_scan3, dim3(bscan), dim3(OCC_SCAN_TPB), 0, st, ctx->occ_bsum, npx, ctx->occ_off,
                           ctx->d_state, first, eval_only);
        hipLaunchKernelGGL(k_occ_scatter, dim3(b256), dim3(256), 0, st, ctx->occ_tgt, npx, ctx->occ_off, ctx->occ_cnt,
                           ctx->occ_list, ctx->d_state, first, eval_only);
        hipLaunchKernelGGL(k_occ_resolve, dim3(b256), dim3(256), 0, st, ctx->occ_off, npx, ctx->occ_list,
                           ctx->occ_dinv, ctx->occ_flags, ctx->d_state, first, eval_only);
        timing_end(ctx, slot);
        R360_HIP(hipGetLastError());
    }
    IcpJobs jobs;
    IcpJob& J = jobs.j[0];
    J.src = Ls.p0; J.trg = Lt.p0; J.tg = Lt.tg; J.pts = Ls.pts; J.npts = src->d_npts + level;
    J.spk = Ls.pk; J.tpk = Lt.pk;
    J.S = ctx->d_state; J.partials = ctx->d_partials; J.gcnt = ctx->d_gticket; J.dq = ctx->d_defer;
    return launch_jobs(ctx, jobs, 1, Ls, T, level, method, C, first, eval_only, G);
}
