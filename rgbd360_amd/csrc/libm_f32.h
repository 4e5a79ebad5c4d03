// libm_f32.h — float asinf / atan2f with the exact arithmetic of the x86-64 glibc the reference
// runs on (the classic fdlibm/Cephes single-precision algorithms of sysdeps/ieee754/flt-32).
//
// Why: the reference projects each point with std::asin(float) / std::atan2(float, float) and then
// rounds to a pixel (RegisterPhotoICP.h:2677-2680, 2978-2981).  glibc's float versions are not
// correctly rounded (7 % / 16 % of random arguments differ from the correctly rounded value), and
// ocml's differ again, so a pixel whose coordinate lands within an ulp of .5 flips between
// implementations.  Evaluating the same polynomial program on the GPU (IEEE div/sqrt,
// -ffp-contract=off) makes the device projection bit-identical to the CPU reference.  The equality
// with the host glibc is checked by tests/test_abi.py::test_libm_port_matches_glibc over millions of
// arguments (and on the GPU by tests/test_gpu_dense.py).
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define R360_HD __host__ __device__ __forceinline__
#else
#define R360_HD inline
#endif

namespace r360m {

R360_HD uint32_t fbits(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
R360_HD float bitsf(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }
R360_HD float fabs_(float x) { return bitsf(fbits(x) & 0x7fffffffu); }

R360_HD float asinf(float x) {
    const float one = 1.0f, huge = 1.0e30f;
    const float pio2_hi = 1.57079637050628662109375f;
    const float pio2_lo = -4.37113900018624283e-8f;
    const float pio4_hi = 0.785398185253143310546875f;
    const float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f, p3 = 2.417951451e-2f,
                p4 = 4.216630880e-2f;
    const int32_t hx = (int32_t)fbits(x);
    const int32_t ix = hx & 0x7fffffff;
    float t, w, p, q, c, r, s;
    if (ix == 0x3f800000) return x * pio2_hi + x * pio2_lo;
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix < 0x3f000000) {
        if (ix < 0x32000000) {
            if (huge + x > one) return x;
        } else {
            t = x * x;
            w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
            return x + x * w;
        }
    }
    w = one - fabs_(x);
    t = w * 0.5f;
    p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    s = sqrtf(t);
    if (ix >= 0x3F79999A) {
        t = pio2_hi - (2.0f * (s + s * p) - pio2_lo);
    } else {
        w = bitsf(fbits(s) & 0xfffff000u);
        c = (t - w * w) / (s + w);
        r = p;
        p = 2.0f * s * r - (pio2_lo - 2.0f * c);
        q = pio4_hi - 2.0f * w;
        t = pio4_hi - (p - q);
    }
    return hx > 0 ? t : -t;
}

R360_HD float atanf(float x) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT[11] = {3.3333334327e-01f, -2.0000000298e-01f, 1.4285714924e-01f, -1.1111110449e-01f,
                          9.0908870101e-02f, -7.6918758452e-02f, 6.6610731184e-02f, -5.8335702866e-02f,
                          4.9768779427e-02f, -3.6531571299e-02f, 1.6285819933e-02f};
    const float one = 1.0f, huge = 1.0e30f;
    const int32_t hx = (int32_t)fbits(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {
        if (ix < 0x31000000) {
            if (huge + x > one) return x;
        }
        id = -1;
    } else {
        x = fabs_(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - one) / (2.0f + x); }
            else { id = 1; x = (x - one) / (x + one); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (one + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    // table entries by selects (an indexed load would be the only memory access of the device path)
    const float hi = id == 0 ? atanhi[0] : (id == 1 ? atanhi[1] : (id == 2 ? atanhi[2] : atanhi[3]));
    const float lo = id == 0 ? atanlo[0] : (id == 1 ? atanlo[1] : (id == 2 ? atanlo[2] : atanlo[3]));
    const float zz = hi - ((x * (s1 + s2) - lo) - x);
    return hx < 0 ? -zz : zz;
}

R360_HD float atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)fbits(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        } else {
            switch (m) {
                case 0: return 0.0f;
                case 1: return -0.0f;
                case 2: return pi + tiny;
                default: return -pi - tiny;
            }
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = atanf(fabs_(y / x));
    switch (m) {
        case 0: return z;
        case 1: return bitsf(fbits(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// ---------------------------------------------------------------------------------------------
// Branch-light forms for the GPU pixel loop: the same arithmetic as atanf/atan2f above (so the same
// bits), with the argument-reduction case chosen by selects and ONE division, so a wave does not
// serialise the five reduction branches.  Special arguments (zeros, infinities, NaN, x == 1,
// |y/x| beyond 2^+-60) take the exact reference path above.
R360_HD float atanf_sel(float x) {
    const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f, atanhi2 = 9.8279368877e-01f,
                atanhi3 = 1.5707962513e+00f;
    const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f, atanlo2 = 3.4473217170e-08f,
                atanlo3 = 7.5497894159e-08f;
    const int32_t hx = (int32_t)fbits(x);
    const int32_t ix = hx & 0x7fffffff;
    const int id = ix < 0x3ee00000 ? -1 : (ix < 0x3f300000 ? 0 : (ix < 0x3f980000 ? 1 : (ix < 0x401c0000 ? 2 : 3)));
    const float ax = fabs_(x);
    const float num = id < 0 ? x : (id == 0 ? 2.0f * ax - 1.0f : (id == 1 ? ax - 1.0f : (id == 2 ? ax - 1.5f : -1.0f)));
    const float den = id < 0 ? 1.0f : (id == 0 ? 2.0f + ax : (id == 1 ? ax + 1.0f : (id == 2 ? 1.0f + 1.5f * ax : ax)));
    const float xr = num / den;  // exact: num/1 == num for id < 0
    const float z = xr * xr;
    const float w = z * z;
    const float s1 = z * (3.3333334327e-01f + w * (1.4285714924e-01f + w * (9.0908870101e-02f +
                     w * (6.6610731184e-02f + w * (4.9768779427e-02f + w * 1.6285819933e-02f)))));
    const float s2 = w * (-2.0000000298e-01f + w * (-1.1111110449e-01f + w * (-7.6918758452e-02f +
                     w * (-5.8335702866e-02f + w * -3.6531571299e-02f))));
    const float hi = id == 0 ? atanhi0 : (id == 1 ? atanhi1 : (id == 2 ? atanhi2 : atanhi3));
    const float lo = id == 0 ? atanlo0 : (id == 1 ? atanlo1 : (id == 2 ? atanlo2 : atanlo3));
    const float zz = hi - ((xr * (s1 + s2) - lo) - xr);
    float res = id < 0 ? xr - xr * (s1 + s2) : (hx < 0 ? -zz : zz);
    if (ix < 0x31000000) res = x;                                    // |x| < 2^-29
    if (ix >= 0x4c000000) res = ix > 0x7f800000 ? x + x : (hx > 0 ? atanhi3 + atanlo3 : -atanhi3 - atanlo3);
    return res;
}

R360_HD float atan2f_sel(float y, float x) {
    const float pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)fbits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)fbits(y), iy = hy & 0x7fffffff;
    const int k = (iy - ix) >> 23;
    const bool special = (ix == 0) | (iy == 0) | (ix >= 0x7f800000) | (iy >= 0x7f800000) | (hx == 0x3f800000) |
                         (k > 60) | (hx < 0 && k < -60);
    if (special) return atan2f(y, x);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    const float z = atanf_sel(fabs_(y / x));
    return m == 0 ? z : (m == 1 ? -z : (m == 2 ? pi - (z - pi_lo) : (z - pi_lo) - pi));
}

// ---------------------------------------------------------------------------------------------
// Fast forms for the GPU projection (NOT bit-exact): the same polynomials with the IEEE division and
// square root replaced by the hardware reciprocal / square root (~1 ulp).  The ICP pass uses them only
// to decide on which side of a pixel-rounding boundary a projection falls; when it lands within the
// guard band of a boundary the exact functions above recompute it (icp_kernels.hip, project()).
#if defined(__HIPCC__)
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }

__device__ __forceinline__ float asinf_fast(float x) {
    const float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f, p3 = 2.417951451e-2f,
                p4 = 4.216630880e-2f;
    const float ax = fabs_(x);
    if (ax < 0.5f) {                                       // the exact polynomial branch
        const float t = x * x;
        return x + x * (t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4)))));
    }
    const float t = (1.0f - ax) * 0.5f;
    const float p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    const float s = fast_sqrt(t);
    const float r = 1.57079637050628662109375f - 2.0f * (s + s * p);
    return x > 0 ? r : -r;
}

// asin for the spherical projection's row decision only: below |x| = 0.53 the |x| < 0.5 polynomial of
// asinf (accurate to 1 ulp up to 0.53), with contraction; at and above it the caller's `out`.  The
// stitched sphere spans |phi| <= 30 deg (H = W / 6, Frame360.h:391-392), so there |x| >= 0.53 (|phi| >= 32
// deg) always projects outside the image at every pyramid level and out = 1 (a row outside as well) is
// exact in effect.  A taller sphere (r360_calib_create_sphere with H > 0.175 W) passes out = NaN: those
// lanes are flagged by the guard test and re-projected exactly (project_exact).
__device__ __forceinline__ float asinf_fast_view(float x, float out = 1.0f) {
#pragma clang fp contract(fast)
    const float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f, p3 = 2.417951451e-2f,
                p4 = 4.216630880e-2f;
    const float t = x * x;
    const float r = x + x * (t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4)))));
    return fabs_(x) < 0.53f ? r : __builtin_copysignf(out, x);
}

// atan2 with a two-way argument reduction (|t| <= tan(pi/8) < 7/16, fdlibm's polynomial domain):
// atan(a) = a poly for a <= tan(pi/8), pi/4 + atan((a-1)/(a+1)) above; octants by selects.
__device__ __forceinline__ float atan2f_fast(float y, float x) {
    const float ay = fabs_(y), ax = fabs_(x);
    const float mx = ay > ax ? ay : ax, mn = ay > ax ? ax : ay;
    const float a = mn * fast_rcp(mx);                     // in [0, 1]
    const bool big = a > 0.41421356f;
    const float t = big ? (a - 1.0f) * fast_rcp(a + 1.0f) : a;
    const float z = t * t, w = z * z;
    const float s1 = z * (3.3333334327e-01f + w * (1.4285714924e-01f + w * (9.0908870101e-02f +
                     w * (6.6610731184e-02f + w * (4.9768779427e-02f + w * 1.6285819933e-02f)))));
    const float s2 = w * (-2.0000000298e-01f + w * (-1.1111110449e-01f + w * (-7.6918758452e-02f +
                     w * (-5.8335702866e-02f + w * -3.6531571299e-02f))));
    float r = t - t * (s1 + s2);
    r = big ? r + 0.78539816f : r;
    r = ay > ax ? 1.57079633f - r : r;
    r = (fbits(x) >> 31) ? 3.14159265f - r : r;
    return (fbits(y) >> 31) ? -r : r;
}

// Correctly rounded f32 square root and division for NORMAL operands and results (no scaling, no
// special-value fix-up): the compiler's own IEEE sequences (v_sqrt + neighbour tests; v_rcp + Newton +
// two fma corrections) without their range handling.  The ICP pass's error terms go through them, so
// they equal the reference's sqrtf / '/' bit for bit (tests/test_gpu_dense.py checks both against the
// compiler's IEEE operations).  sqrt_rn(0) = 0.
__device__ __forceinline__ float sqrt_rn(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float vm = __builtin_fmaf(-sm, s, x), vp = __builtin_fmaf(-sp, s, x);
    float r = vm <= 0.f ? sm : s;
    r = vp > 0.f ? sp : r;
    return r;
}
__device__ __forceinline__ float div_rn(float a, float b) {
    float r = __builtin_amdgcn_rcpf(b);
    r = __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
    float q = a * r;
    q = __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
    return __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
}

// atan2 as atan2f_fast with a single reciprocal: the reduction t = (mn - mx) / (mn + mx) above
// tan(pi/8) (= (a - 1) / (a + 1) for a = mn / mx) and t = mn / mx below share one division.
__device__ __forceinline__ float atan2f_fast1(float y, float x) {
#pragma clang fp contract(fast)
    const float ay = fabs_(y), ax = fabs_(x);
    const float mx = ay > ax ? ay : ax, mn = ay > ax ? ax : ay;
    const bool big = mn > 0.41421356f * mx;
    const float t = (big ? mn - mx : mn) * fast_rcp(big ? mn + mx : mx);
    // atan(t) = t + t z P(z), z = t^2, |t| <= tan(pi/8): a 5-term fit (round 4; fdlibm's 11 terms are made for
    // |t| <= 7/16 at full float accuracy).  Float evaluation within 1.9e-8 rad of atan over the domain, far inside
    // the projection's guard band (1.5e-3 px = 2.5e-6 rad at level 0 of a 3840-column sphere); the exact path
    // decides every lane inside the band (tests/test_gpu_dense.py checks fast vs exact decisions).
    const float z = t * t;
    const float p = -3.3333301544e-01f + z * (1.9997815788e-01f + z * (-1.4233337343e-01f +
                    z * (1.0528898239e-01f + z * -5.9325449169e-02f)));
    float r = t + (t * z) * p;
    r = big ? r + 0.78539816f : r;
    r = ay > ax ? 1.57079633f - r : r;
    r = (fbits(x) >> 31) ? 3.14159265f - r : r;
    return __builtin_copysignf(r, y);   // r >= 0
}
#endif

}  // namespace r360m
