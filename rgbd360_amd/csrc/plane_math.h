// plane_math.h — arithmetic of the plane half shared by the HIP kernels and the host runtime of
// librgbd360_hip.so (never by the oracle, which restates the same definitions independently).
//
//  * Exact point-set moments: coordinates are quantised to q = (int64)(v * 2^36) (exact for every
//    back-projected coordinate, |v| >= 2^-13), first moments are summed in int64 and second moments in
//    int128, so sums are order-free and a parallel reduction reproduces a sequential one bit for bit.
//    cov = (n Sxy - Sx Sy) / n^2 is formed in int128 and rounded once.
//  * pcl::eigen33 (smallest eigenpair of a symmetric 3x3, float), with std::atan2 as glibc's atan2f
//    (libm_f32.h) and std::cos/std::sin as fixed double Taylor polynomials rounded to float.
#pragma once
#include <stdint.h>
#include "libm_f32.h"

namespace r360p {

typedef __int128 i128;

R360_HD long long q36(float v) { return (long long)((double)v * 68719476736.0); }

R360_HD double i128_to_double(i128 v) {
    const bool neg = v < 0;
    const unsigned __int128 u = neg ? -(unsigned __int128)v : (unsigned __int128)v;
    const double d = (double)(unsigned long long)(u >> 64) * 18446744073709551616.0 + (double)(unsigned long long)u;
    return neg ? -d : d;
}

// Raw moment sums of a point set (+ colour sums for the plane descriptors).
struct Moments {
    long long n;
    long long s1[3];
    i128 s2[6];            // xx xy xz yy yz zz
    long long c[4];        // sum r/(r+g+b), g/., b/. in 2^-33 fixed point; sum of r+g+b
};

R360_HD void moments_zero(Moments& m) {
    m.n = 0;
    for (int k = 0; k < 3; ++k) m.s1[k] = 0;
    for (int k = 0; k < 6; ++k) m.s2[k] = 0;
    for (int k = 0; k < 4; ++k) m.c[k] = 0;
}

R360_HD void moments_add_xyz(Moments& m, float x, float y, float z) {
    const long long q[3] = {q36(x), q36(y), q36(z)};
    m.n += 1;
    for (int k = 0; k < 3; ++k) m.s1[k] += q[k];
    m.s2[0] += (i128)q[0] * q[0];
    m.s2[1] += (i128)q[0] * q[1];
    m.s2[2] += (i128)q[0] * q[2];
    m.s2[3] += (i128)q[1] * q[1];
    m.s2[4] += (i128)q[1] * q[2];
    m.s2[5] += (i128)q[2] * q[2];
}

R360_HD void moments_add_rgb(Moments& m, uint8_t r, uint8_t g, uint8_t b) {
    const int sum = r + g + b;
    if (sum != 0) {
        const float inv = 1.0f / float(sum);
        m.c[0] += (long long)((double)(float(r) * inv) * 8589934592.0);
        m.c[1] += (long long)((double)(float(g) * inv) * 8589934592.0);
        m.c[2] += (long long)((double)(float(b) * inv) * 8589934592.0);
    }
    m.c[3] += sum;
}

R360_HD void moments_merge(Moments& a, const Moments& b) {
    a.n += b.n;
    for (int k = 0; k < 3; ++k) a.s1[k] += b.s1[k];
    for (int k = 0; k < 6; ++k) a.s2[k] += b.s2[k];
    for (int k = 0; k < 4; ++k) a.c[k] += b.c[k];
}

// mean (double) and covariance (double, row-major), normalised by n
R360_HD void moments_mean_cov(const Moments& m, double mean[3], double cov[9]) {
    const double dn = (double)m.n;
    for (int k = 0; k < 3; ++k) mean[k] = ((double)m.s1[k] * 1.4551915228366852e-11) / dn;   // 2^-36
    int t = 0;
    for (int a = 0; a < 3; ++a)
        for (int b = a; b < 3; ++b, ++t) {
            const i128 num = (i128)m.n * m.s2[t] - (i128)m.s1[a] * m.s1[b];
            const double c = i128_to_double(num) * 2.117582368135751e-22 / (dn * dn);          // 2^-72
            cov[a * 3 + b] = c;
            cov[b * 3 + a] = c;
        }
}

// ---------------------------------------------------------------- pcl::eigen33 (float)
R360_HD float sin_poly(float xf) {
    const double x = xf, x2 = x * x;
    double p = 1.0 / 355687428096000.0;
    p = p * x2 - 1.0 / 1307674368000.0;
    p = p * x2 + 1.0 / 6227020800.0;
    p = p * x2 - 1.0 / 39916800.0;
    p = p * x2 + 1.0 / 362880.0;
    p = p * x2 - 1.0 / 5040.0;
    p = p * x2 + 1.0 / 120.0;
    p = p * x2 - 1.0 / 6.0;
    p = p * x2 + 1.0;
    return float(p * x);
}
R360_HD float cos_poly(float xf) {
    const double x = xf, x2 = x * x;
    double p = 1.0 / 6402373705728000.0;
    p = p * x2 - 1.0 / 20922789888000.0;
    p = p * x2 + 1.0 / 87178291200.0;
    p = p * x2 - 1.0 / 479001600.0;
    p = p * x2 + 1.0 / 3628800.0;
    p = p * x2 - 1.0 / 40320.0;
    p = p * x2 + 1.0 / 720.0;
    p = p * x2 - 1.0 / 24.0;
    p = p * x2 + 0.5;
    p = p * x2;
    return float(1.0 - p);
}

R360_HD void swapf(float& a, float& b) { const float t = a; a = b; b = t; }

R360_HD void compute_roots2(float b, float c, float roots[3]) {
    roots[0] = 0.f;
    float d = float(b * b - 4.0 * c);
    if (d < 0.0) d = 0.0;
    const float sd = sqrtf(d);
    roots[2] = 0.5f * (b + sd);
    roots[1] = 0.5f * (b - sd);
}

// m: symmetric 3x3, column-major
R360_HD void compute_roots(const float m[9], float roots[3]) {
#define M_(r, c) m[(c) * 3 + (r)]
    const float c0 = M_(0, 0) * M_(1, 1) * M_(2, 2) + float(2) * M_(0, 1) * M_(0, 2) * M_(1, 2) -
                     M_(0, 0) * M_(1, 2) * M_(1, 2) - M_(1, 1) * M_(0, 2) * M_(0, 2) - M_(2, 2) * M_(0, 1) * M_(0, 1);
    const float c1 = M_(0, 0) * M_(1, 1) - M_(0, 1) * M_(0, 1) + M_(0, 0) * M_(2, 2) - M_(0, 2) * M_(0, 2) +
                     M_(1, 1) * M_(2, 2) - M_(1, 2) * M_(1, 2);
    const float c2 = M_(0, 0) + M_(1, 1) + M_(2, 2);
#undef M_
    if (r360m::fabs_(c0) < 1.1920928955078125e-07f) {
        compute_roots2(c2, c1, roots);
        return;
    }
    const float s_inv3 = float(1.0 / 3.0);
    const float s_sqrt3 = sqrtf(float(3.0));
    const float c2_over_3 = c2 * s_inv3;
    float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
    if (a_over_3 > float(0)) a_over_3 = float(0);
    const float half_b = float(0.5) * (c0 + c2_over_3 * (float(2) * c2_over_3 * c2_over_3 - c1));
    float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
    if (q > float(0)) q = float(0);
    const float rho = sqrtf(-a_over_3);
    const float theta = r360m::atan2f(sqrtf(-q), half_b) * s_inv3;
    const float cos_theta = cos_poly(theta);
    const float sin_theta = sin_poly(theta);
    roots[0] = c2_over_3 + float(2) * rho * cos_theta;
    roots[1] = c2_over_3 - rho * (cos_theta + s_sqrt3 * sin_theta);
    roots[2] = c2_over_3 - rho * (cos_theta - s_sqrt3 * sin_theta);
    if (roots[0] >= roots[1]) swapf(roots[0], roots[1]);
    if (roots[1] >= roots[2]) {
        swapf(roots[1], roots[2]);
        if (roots[0] >= roots[1]) swapf(roots[0], roots[1]);
    }
    if (roots[0] <= 0) compute_roots2(c2, c1, roots);
}

R360_HD void eigen33_min(const float mat[9], float& eigenvalue, float ev[3]) {
    float scale = 0.f;
    for (int i = 0; i < 9; ++i) {
        const float a = r360m::fabs_(mat[i]);
        scale = scale < a ? a : scale;
    }
    if (scale <= 1.17549435e-38f) scale = 1.0f;
    float s[9];
    for (int i = 0; i < 9; ++i) s[i] = mat[i] / scale;
    float roots[3];
    compute_roots(s, roots);
    eigenvalue = roots[0] * scale;
    for (int k = 0; k < 3; ++k) s[k * 3 + k] -= roots[0];
    const float r0[3] = {s[0], s[3], s[6]}, r1[3] = {s[1], s[4], s[7]}, r2[3] = {s[2], s[5], s[8]};
    float v1[3], v2[3], v3[3];
    v1[0] = r0[1] * r1[2] - r0[2] * r1[1]; v1[1] = r0[2] * r1[0] - r0[0] * r1[2]; v1[2] = r0[0] * r1[1] - r0[1] * r1[0];
    v2[0] = r0[1] * r2[2] - r0[2] * r2[1]; v2[1] = r0[2] * r2[0] - r0[0] * r2[2]; v2[2] = r0[0] * r2[1] - r0[1] * r2[0];
    v3[0] = r1[1] * r2[2] - r1[2] * r2[1]; v3[1] = r1[2] * r2[0] - r1[0] * r2[2]; v3[2] = r1[0] * r2[1] - r1[1] * r2[0];
    const float l1 = v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2];
    const float l2 = v2[0] * v2[0] + v2[1] * v2[1] + v2[2] * v2[2];
    const float l3 = v3[0] * v3[0] + v3[1] * v3[1] + v3[2] * v3[2];
    const float* v;
    float l;
    if (l1 >= l2 && l1 >= l3) { v = v1; l = l1; }
    else if (l2 >= l1 && l2 >= l3) { v = v2; l = l2; }
    else { v = v3; l = l3; }
    const float sl = sqrtf(l);
    for (int k = 0; k < 3; ++k) ev[k] = v[k] / sl;
}

// Eigen Vector4f dot on x86-64 SSE (packet product + movehl horizontal add)
R360_HD float dot4(const float a[4], const float b[4]) {
    const float p0 = a[0] * b[0], p1 = a[1] * b[1], p2 = a[2] * b[2], p3 = a[3] * b[3];
    return (p0 + p2) + (p1 + p3);
}

}  // namespace r360p
