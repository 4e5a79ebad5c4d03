// planes_oracle.cpp — CPU ORACLE (test infrastructure only) for the per-pixel stages of the plane
// half: cloud back-projection + 2x2 median downsample (A3), fast bilateral filter (A4), integral-image
// normals (A6) and organized multi-plane segmentation with refinement and boundary tracing (A7).
//
// A3 restates vendored reference code line by line.  A4/A6/A7 are PCL 1.7 algorithms the reference
// calls but does not vendor (Frame360.h:493-499, 945-977); they are restated from SURVEY.md App. C
// and the published PCL 1.7 sources (fast_bilateral.hpp, integral_image_normal.hpp,
// integral_image2D.hpp, organized_connected_component_segmentation.hpp,
// organized_multi_plane_segmentation.hpp, plane_coefficient_comparator.h,
// plane_refinement_comparator.h, centroid.hpp, eigen.hpp).  PCL is unpinned:
// "parity unpinned" for these stages.  Documented choices where PCL versions differ:
//   * OrganizedConnectedComponentSegmentation registers a new run with its OWN id (the later,
//     fixed PCL form; the oldest form pushed the row-start label, which is undefined behaviour when
//     that pixel is invalid).
//   * the depth-change test uses fabsf (std::abs on float).
//   * per-label mean/covariance are EXACT: coordinates are quantised to q = (int64)(v * 2^36) (exact
//     for |v| >= 2^-13, which every back-projected coordinate satisfies), first moments are summed in
//     int64 and second moments in int128, cov = (n*Sxy - Sx*Sy) / n^2 is formed in int128 and rounded
//     once.  PCL 1.7 sums in float in raster order, an order no parallel reduction can reproduce;
//     exact sums are order-free, so the GPU reproduces them bit for bit (moments_t below).
//   * eigen33's std::cos/std::sin(float) are evaluated as a fixed double Taylor polynomial rounded to
//     float (glibc's sinf/cosf are not portable to the GPU); std::atan2(float) is glibc's.
//   * the refinement comparator's threshold is the constant 0.02 m (depth_dependent_ = false).
#include "oracle360.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

namespace {
const float kNaN = std::numeric_limits<float>::quiet_NaN();

inline bool isfin(float v) { return std::isfinite(v); }
}  // namespace

// Exact moments of a point set (see header).  Shared by the segmentation fit and the plane
// descriptors (pbmap_oracle.cpp).
namespace orc_moments {
typedef __int128 i128;
long long q36(float v) { return (long long)((double)v * 68719476736.0); }
double i128_to_double(i128 v) {
    const bool neg = v < 0;
    unsigned __int128 u = neg ? -(unsigned __int128)v : (unsigned __int128)v;
    const double d = (double)(unsigned long long)(u >> 64) * 18446744073709551616.0 + (double)(unsigned long long)u;
    return neg ? -d : d;
}
struct Moments {
    long long n = 0;
    long long s1[3] = {0, 0, 0};
    i128 s2[6] = {0, 0, 0, 0, 0, 0};  // xx xy xz yy yz zz
    void add(float x, float y, float z) {
        const long long q[3] = {q36(x), q36(y), q36(z)};
        ++n;
        for (int k = 0; k < 3; ++k) s1[k] += q[k];
        int t = 0;
        for (int a = 0; a < 3; ++a)
            for (int b = a; b < 3; ++b) s2[t++] += (i128)q[a] * q[b];
    }
    void merge(const Moments& o) {
        n += o.n;
        for (int k = 0; k < 3; ++k) s1[k] += o.s1[k];
        for (int k = 0; k < 6; ++k) s2[k] += o.s2[k];
    }
    // mean (double) and covariance (double, row-major 3x3), normalised by n
    void mean_cov(double mean[3], double cov[9]) const {
        const double dn = (double)n;
        for (int k = 0; k < 3; ++k) mean[k] = ((double)s1[k] * 1.4551915228366852e-11) / dn;  // 2^-36
        int t = 0;
        for (int a = 0; a < 3; ++a)
            for (int b = a; b < 3; ++b, ++t) {
                const i128 num = (i128)n * s2[t] - (i128)s1[a] * s1[b];
                const double c = i128_to_double(num) * 2.117582368135751e-22 / (dn * dn);  // 2^-72
                cov[a * 3 + b] = cov[b * 3 + a] = c;
            }
    }
};
}  // namespace orc_moments

// ------------------------------------------------------------------------------------------ A3
// CloudRGBD_Ext.h:78-139 then DownsampleRGBD.h:209-311 (downsamplingStep 2, minDepth 0.3 /
// maxDepth 5.0 of DownsampleRGBD, validity 0.3 <= z <= 10 of CloudRGBD.h:66-67).
extern "C" void orc_cloud_downsample(const float* depth_m, const uint8_t* bgr, int rows, int cols,
                                     float* xyz4, uint8_t* rgb4) {
    const int height = rows, width = cols;
    const float res_factor_VGA = width / 640.0;             // :97
    const float focal_length = 525 * res_factor_VGA;        // :98
    const float inv_fx = 1.f / focal_length, inv_fy = 1.f / focal_length;
    const float ox = width / 2 - 0.5;                        // :101 (int division first)
    const float oy = height / 2 - 0.5;
    std::vector<float> px(size_t(width) * height), py(px.size()), pz(px.size());
    for (int y = 0; y < height; y++)
        for (int x = 0; x < width; x++) {
            const size_t i = size_t(width) * y + x;
            const float z = depth_m[i];
            if (z > 0 && z >= 0.3f && z <= 10.0f) {          // :118
                px[i] = (x - ox) * z * inv_fx;
                py[i] = (y - oy) * z * inv_fy;
                pz[i] = z;
            } else {
                px[i] = py[i] = pz[i] = kNaN;
            }
        }
    const int step = 2, W2 = width / step;
    const float minD = 0.3f, maxD = 5.0f;
    int j = 0;
    for (int r = 0; r < height; r += step)
        for (int c = 0; c < width; c += step, ++j) {
            double xV[4], yV[4], zV[4];
            int n = 0;
            const size_t center = size_t(r + step / 2) * width + c + step / 2;   // :240
            for (int r2 = r; r2 < r + step; r2++)
                for (int c2 = c; c2 < c + step; c2++) {
                    const size_t i = size_t(r2) * width + c2;
                    if (isfin(px[i]) && minD < pz[i] && pz[i] < maxD) {         // :251-256
                        xV[n] = px[i]; yV[n] = py[i]; zV[n] = pz[i]; n++;
                    }
                }
            float* o = xyz4 + 4 * size_t(j);
            uint8_t* oc = rgb4 + 4 * size_t(j);
            const uint8_t* b = bgr + 3 * center;
            oc[0] = b[2]; oc[1] = b[1]; oc[2] = b[0]; oc[3] = 0;   // CloudRGBD_Ext.h:110-113
            if (n > 0) {                                            // upper median, :271-282
                std::sort(xV, xV + n); std::sort(yV, yV + n); std::sort(zV, zV + n);
                o[0] = (float)xV[n / 2]; o[1] = (float)yV[n / 2]; o[2] = (float)zV[n / 2];
            } else {                                                // copy the centre point, :293-300
                o[0] = px[center]; o[1] = py[center]; o[2] = pz[center];
            }
            o[3] = 0.f;
        }
    (void)W2;
}

// ------------------------------------------------------------------------------------------ A4
// pcl::FastBilateralFilter<PointXYZRGBA>::applyFilter (early_division_ = false), sigma_s 10,
// sigma_r 0.05.  Only z changes; non-finite z first becomes the max finite z.
extern "C" void orc_bilateral(float* xyz4, int w, int h) {
    const float sigma_s = 10.0f, sigma_r = 0.05f;
    auto Z = [&](int x, int y) -> float& { return xyz4[4 * (size_t(y) * w + x) + 2]; };
    float base_max = -std::numeric_limits<float>::max(), base_min = std::numeric_limits<float>::max();
    bool found = false;
    for (int x = 0; x < w; ++x)
        for (int y = 0; y < h; ++y)
            if (isfin(Z(x, y))) {
                if (base_max < Z(x, y)) base_max = Z(x, y);
                if (base_min > Z(x, y)) base_min = Z(x, y);
                found = true;
            }
    if (!found) return;
    for (int x = 0; x < w; ++x)
        for (int y = 0; y < h; ++y)
            if (!isfin(Z(x, y))) Z(x, y) = base_max;
    const float base_delta = base_max - base_min;
    const size_t pad = 2;
    const size_t sw = size_t(float(w - 1) / sigma_s) + 1 + 2 * pad;
    const size_t sh = size_t(float(h - 1) / sigma_s) + 1 + 2 * pad;
    const size_t sd = size_t(base_delta / sigma_r) + 1 + 2 * pad;
    // Array3D: v[(x + sw*y)*sd + z], two floats per cell
    std::vector<float> data(sw * sh * sd * 2, 0.f), buf(data.size(), 0.f);
    auto cell = [&](std::vector<float>& a, size_t x, size_t y, size_t z) { return &a[((x + sw * y) * sd + z) * 2]; };
    for (int x = 0; x < w; ++x) {
        const size_t sx = size_t(float(x) / sigma_s + 0.5f) + pad;
        for (int y = 0; y < h; ++y) {
            const float z = Z(x, y) - base_min;
            const size_t sy = size_t(float(y) / sigma_s + 0.5f) + pad;
            const size_t sz = size_t(z / sigma_r + 0.5f) + pad;
            float* d = cell(data, sx, sy, sz);
            d[0] += Z(x, y);
            d[1] += 1.0f;
        }
    }
    const long off[3] = {long(sd), long(sw * sd), 1};
    for (int dim = 0; dim < 3; ++dim)
        for (int it = 0; it < 2; ++it) {
            std::swap(buf, data);
            for (size_t x = 1; x + 1 < sw; ++x)
                for (size_t y = 1; y + 1 < sh; ++y)
                    for (size_t z = 1; z + 1 < sd; ++z) {
                        const long p = long(((x + sw * y) * sd + z) * 2);
                        const long o = off[dim] * 2;
                        for (int k = 0; k < 2; ++k)
                            data[p + k] = (buf[p - o + k] + buf[p + o + k] + 2.0f * buf[p + k]) / 4.0f;
                    }
        }
    auto clampi = [](long v, long lo, long hi) { return v < lo ? lo : (v > hi ? hi : v); };
    for (int x = 0; x < w; ++x)
        for (int y = 0; y < h; ++y) {
            const float z = Z(x, y) - base_min;
            const float fx = float(x) / sigma_s + float(pad), fy = float(y) / sigma_s + float(pad),
                        fz = z / sigma_r + float(pad);
            const long xi = clampi(long(size_t(fx)), 0, long(sw) - 1), xxi = clampi(xi + 1, 0, long(sw) - 1);
            const long yi = clampi(long(size_t(fy)), 0, long(sh) - 1), yyi = clampi(yi + 1, 0, long(sh) - 1);
            const long zi = clampi(long(size_t(fz)), 0, long(sd) - 1), zzi = clampi(zi + 1, 0, long(sd) - 1);
            const float xa = fx - float(xi), ya = fy - float(yi), za = fz - float(zi);
            float D[2];
            for (int k = 0; k < 2; ++k) {
                auto v = [&](long a, long b, long c) { return cell(data, a, b, c)[k]; };
                D[k] = (1.0f - xa) * (1.0f - ya) * (1.0f - za) * v(xi, yi, zi) +
                       xa * (1.0f - ya) * (1.0f - za) * v(xxi, yi, zi) +
                       (1.0f - xa) * ya * (1.0f - za) * v(xi, yyi, zi) +
                       xa * ya * (1.0f - za) * v(xxi, yyi, zi) +
                       (1.0f - xa) * (1.0f - ya) * za * v(xi, yi, zzi) +
                       xa * (1.0f - ya) * za * v(xxi, yi, zzi) +
                       (1.0f - xa) * ya * za * v(xi, yyi, zzi) +
                       xa * ya * za * v(xxi, yyi, zzi);
            }
            Z(x, y) = D[0] / D[1];
        }
}

// ------------------------------------------------------------------------------------------ A6
// IntegralImageNormalEstimation: computeFeature (depth-change map, distance map), initData /
// initAverage3DGradientMethod (central differences), IntegralImage2D<float,3> (double sums + finite
// counts), computeFeatureFull (BORDER_POLICY_IGNORE, depth-dependent smoothing) and
// computePointNormal (AVERAGE_3D_GRADIENT).
extern "C" void orc_normals(const float* xyz4, int w, int h, float* nrm4, float* dist) {
    const size_t N = size_t(w) * h;
    auto P = [&](size_t i, int k) { return xyz4[4 * i + k]; };
    const float max_depth_change_factor = 0.02f, normal_smoothing_size = 8.0f;
    // depth-change map
    std::vector<unsigned char> dcm(N, 255);
    for (int ri = 0; ri < h - 1; ++ri)
        for (int ci = 0; ci < w - 1; ++ci) {
            const size_t index = size_t(ri) * w + ci;
            const float depth = P(index, 2), depthR = P(index + 1, 2), depthD = P(index + w, 2);
            const float ddc = max_depth_change_factor * (fabsf(depth) + 1.0f) * 2.0f;
            if (fabsf(depth - depthR) > ddc || !isfin(depth) || !isfin(depthR)) {
                dcm[index] = 0; dcm[index + 1] = 0;
            }
            if (fabsf(depth - depthD) > ddc || !isfin(depth) || !isfin(depthD)) {
                dcm[index] = 0; dcm[index + w] = 0;
            }
        }
    // distance map: two chamfer passes over the flat array (the row-end reads wrap into the
    // neighbouring row exactly as PCL's pointer arithmetic does)
    for (size_t i = 0; i < N; ++i) dist[i] = dcm[i] == 0 ? 0.0f : float(w + h);
    for (int ri = 1; ri < h; ++ri)
        for (int ci = 1; ci < w; ++ci) {
            float* prev = dist + size_t(ri - 1) * w;
            float* cur = dist + size_t(ri) * w;
            const float upLeft = prev[ci - 1] + 1.4f, up = prev[ci] + 1.0f, upRight = prev[ci + 1] + 1.4f;
            const float left = cur[ci - 1] + 1.0f, center = cur[ci];
            const float m = std::min(std::min(upLeft, up), std::min(left, upRight));
            if (m < center) cur[ci] = m;
        }
    for (int ri = h - 2; ri >= 0; --ri)
        for (int ci = w - 2; ci >= 0; --ci) {
            float* next = dist + size_t(ri + 1) * w;
            float* cur = dist + size_t(ri) * w;
            const float lowerLeft = next[ci - 1] + 1.4f, lower = next[ci] + 1.0f, lowerRight = next[ci + 1] + 1.4f;
            const float right = cur[ci + 1] + 1.0f, center = cur[ci];
            const float m = std::min(std::min(lowerLeft, lower), std::min(right, lowerRight));
            if (m < center) cur[ci] = m;
        }
    // central differences (interior pixels), zero elsewhere
    std::vector<float> dx(N * 3, 0.f), dy(N * 3, 0.f);
    for (int ri = 1; ri < h - 1; ++ri)
        for (int ci = 1; ci < w - 1; ++ci) {
            const size_t i = size_t(ri) * w + ci;
            for (int k = 0; k < 3; ++k) {
                dx[3 * i + k] = P(i + 1, k) - P(i - 1, k);
                dy[3 * i + k] = P(i + w, k) - P(i - w, k);
            }
        }
    // integral images (w+1) x (h+1), double sums over elements whose x+y+z is finite
    const size_t W1 = size_t(w) + 1;
    std::vector<double> IX((h + 1) * W1 * 3, 0.0), IY(IX.size(), 0.0);
    std::vector<unsigned> CX((h + 1) * W1, 0), CY(CX.size(), 0);
    auto integrate = [&](const std::vector<float>& d, std::vector<double>& I, std::vector<unsigned>& C) {
        for (int r = 0; r < h; ++r)
            for (int c = 0; c < w; ++c) {
                const size_t o = (r + 1) * W1 + c + 1, up = r * W1 + c + 1, lf = (r + 1) * W1 + c, ul = r * W1 + c;
                for (int k = 0; k < 3; ++k) I[3 * o + k] = I[3 * up + k] + I[3 * lf + k] - I[3 * ul + k];
                C[o] = C[up] + C[lf] - C[ul];
                const float* e = &d[3 * (size_t(r) * w + c)];
                if (isfin(e[0] + e[1] + e[2])) {
                    for (int k = 0; k < 3; ++k) I[3 * o + k] += double(e[k]);
                    ++C[o];
                }
            }
    };
    integrate(dx, IX, CX);
    integrate(dy, IY, CY);
    auto rect_sum = [&](const std::vector<double>& I, int sx, int sy, int rw, int rh, double out[3]) {
        const size_t ul = size_t(sy) * W1 + sx, ur = ul + rw, ll = size_t(sy + rh) * W1 + sx, lr = ll + rw;
        for (int k = 0; k < 3; ++k) out[k] = I[3 * lr + k] + I[3 * ul + k] - I[3 * ur + k] - I[3 * ll + k];
    };
    auto rect_cnt = [&](const std::vector<unsigned>& C, int sx, int sy, int rw, int rh) {
        const size_t ul = size_t(sy) * W1 + sx, ur = ul + rw, ll = size_t(sy + rh) * W1 + sx, lr = ll + rw;
        return C[lr] + C[ul] - C[ur] - C[ll];
    };
    for (size_t i = 0; i < N; ++i) { nrm4[4 * i] = nrm4[4 * i + 1] = nrm4[4 * i + 2] = kNaN; nrm4[4 * i + 3] = 0.f; }
    const int border = int(normal_smoothing_size);
    for (int ri = border; ri < h - border; ++ri)
        for (int ci = border; ci < w - border; ++ci) {
            const size_t index = size_t(ri) * w + ci;
            const float depth = P(index, 2);
            if (!isfin(depth)) continue;
            const float smoothing = std::min(dist[index], normal_smoothing_size + depth / 10.0f);
            if (!(smoothing > 2.0f)) continue;
            const int rw = int(smoothing), rh = int(smoothing), rw2 = rw / 2, rh2 = rh / 2;
            const int sx = ci - rw2, sy = ri - rh2;
            if (rect_cnt(CX, sx, sy, rw, rh) == 0 || rect_cnt(CY, sx, sy, rw, rh) == 0) continue;
            double gx[3], gy[3];
            rect_sum(IX, sx, sy, rw, rh, gx);
            rect_sum(IY, sx, sy, rw, rh, gy);
            double n[3] = {gy[1] * gx[2] - gy[2] * gx[1], gy[2] * gx[0] - gy[0] * gx[2], gy[0] * gx[1] - gy[1] * gx[0]};
            const double len = n[0] * n[0] + n[1] * n[1] + n[2] * n[2];
            if (len == 0.0) continue;
            const double s = std::sqrt(len);
            float nx = float(n[0] / s), ny = float(n[1] / s), nz = float(n[2] / s);
            // flipNormalTowardsViewpoint, viewpoint (0,0,0)
            const float vx = 0.f - P(index, 0), vy = 0.f - P(index, 1), vz = 0.f - P(index, 2);
            const float cos_theta = vx * nx + vy * ny + vz * nz;
            if (cos_theta < 0) { nx *= -1; ny *= -1; nz *= -1; }
            nrm4[4 * index] = nx; nrm4[4 * index + 1] = ny; nrm4[4 * index + 2] = nz;
        }
}

// ------------------------------------------------------------------------------------------ A7
namespace {

// cos/sin of eigen33 (theta in [0, pi/3]): Taylor polynomials in double (Horner, no FMA), rounded to
// float once; the device evaluates the identical expression.
float sin_poly(float xf) {
    const double x = xf, x2 = x * x;
    double p = 1.0 / 355687428096000.0;                    // 1/17!
    p = p * x2 - 1.0 / 1307674368000.0;                    // 1/15!
    p = p * x2 + 1.0 / 6227020800.0;                       // 1/13!
    p = p * x2 - 1.0 / 39916800.0;                         // 1/11!
    p = p * x2 + 1.0 / 362880.0;                           // 1/9!
    p = p * x2 - 1.0 / 5040.0;
    p = p * x2 + 1.0 / 120.0;
    p = p * x2 - 1.0 / 6.0;
    p = p * x2 + 1.0;
    return float(p * x);
}
float cos_poly(float xf) {
    const double x = xf, x2 = x * x;
    double p = 1.0 / 6402373705728000.0;                   // 1/18!
    p = p * x2 - 1.0 / 20922789888000.0;                   // 1/16!
    p = p * x2 + 1.0 / 87178291200.0;                      // 1/14!
    p = p * x2 - 1.0 / 479001600.0;                        // 1/12!
    p = p * x2 + 1.0 / 3628800.0;                          // 1/10!
    p = p * x2 - 1.0 / 40320.0;
    p = p * x2 + 1.0 / 720.0;
    p = p * x2 - 1.0 / 24.0;
    p = p * x2 + 0.5;
    p = p * x2;
    return float(1.0 - p);
}

// pcl::eigen33 smallest eigenpair (pcl/common/eigen.hpp: computeRoots2, computeRoots, eigen33)
void compute_roots2(float b, float c, float roots[3]) {
    roots[0] = 0.f;
    float d = float(b * b - 4.0 * c);
    if (d < 0.0) d = 0.0;
    const float sd = std::sqrt(d);
    roots[2] = 0.5f * (b + sd);
    roots[1] = 0.5f * (b - sd);
}

void compute_roots(const float m[9], float roots[3]) {
    auto M = [&](int r, int c) { return m[c * 3 + r]; };
    const float c0 = M(0, 0) * M(1, 1) * M(2, 2) + float(2) * M(0, 1) * M(0, 2) * M(1, 2) -
                     M(0, 0) * M(1, 2) * M(1, 2) - M(1, 1) * M(0, 2) * M(0, 2) - M(2, 2) * M(0, 1) * M(0, 1);
    const float c1 = M(0, 0) * M(1, 1) - M(0, 1) * M(0, 1) + M(0, 0) * M(2, 2) - M(0, 2) * M(0, 2) +
                     M(1, 1) * M(2, 2) - M(1, 2) * M(1, 2);
    const float c2 = M(0, 0) + M(1, 1) + M(2, 2);
    if (std::fabs(c0) < std::numeric_limits<float>::epsilon()) {
        compute_roots2(c2, c1, roots);
        return;
    }
    const float s_inv3 = float(1.0 / 3.0);
    const float s_sqrt3 = std::sqrt(float(3.0));
    const float c2_over_3 = c2 * s_inv3;
    float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
    if (a_over_3 > float(0)) a_over_3 = float(0);
    const float half_b = float(0.5) * (c0 + c2_over_3 * (float(2) * c2_over_3 * c2_over_3 - c1));
    float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
    if (q > float(0)) q = float(0);
    const float rho = std::sqrt(-a_over_3);
    const float theta = std::atan2(std::sqrt(-q), half_b) * s_inv3;
    const float cos_theta = cos_poly(theta);
    const float sin_theta = sin_poly(theta);
    roots[0] = c2_over_3 + float(2) * rho * cos_theta;
    roots[1] = c2_over_3 - rho * (cos_theta + s_sqrt3 * sin_theta);
    roots[2] = c2_over_3 - rho * (cos_theta - s_sqrt3 * sin_theta);
    if (roots[0] >= roots[1]) std::swap(roots[0], roots[1]);
    if (roots[1] >= roots[2]) {
        std::swap(roots[1], roots[2]);
        if (roots[0] >= roots[1]) std::swap(roots[0], roots[1]);
    }
    if (roots[0] <= 0) compute_roots2(c2, c1, roots);
}

void eigen33_min(const float mat[9], float& eigenvalue, float ev[3]) {
    float scale = 0.f;
    for (int i = 0; i < 9; ++i) scale = std::max(scale, std::fabs(mat[i]));
    if (scale <= std::numeric_limits<float>::min()) scale = 1.0f;
    float s[9];
    for (int i = 0; i < 9; ++i) s[i] = mat[i] / scale;
    float roots[3];
    compute_roots(s, roots);
    eigenvalue = roots[0] * scale;
    for (int k = 0; k < 3; ++k) s[k * 3 + k] -= roots[0];
    auto row = [&](int r, float o[3]) { o[0] = s[r]; o[1] = s[3 + r]; o[2] = s[6 + r]; };
    float r0[3], r1[3], r2[3];
    row(0, r0); row(1, r1); row(2, r2);
    auto cross = [](const float a[3], const float b[3], float o[3]) {
        o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0];
    };
    float v1[3], v2[3], v3[3];
    cross(r0, r1, v1); cross(r0, r2, v2); cross(r1, r2, v3);
    auto sq = [](const float v[3]) { return v[0] * v[0] + v[1] * v[1] + v[2] * v[2]; };
    const float l1 = sq(v1), l2 = sq(v2), l3 = sq(v3);
    const float* v;
    float l;
    if (l1 >= l2 && l1 >= l3) { v = v1; l = l1; }
    else if (l2 >= l1 && l2 >= l3) { v = v2; l = l2; }
    else { v = v3; l = l3; }
    const float sl = std::sqrt(l);
    for (int k = 0; k < 3; ++k) ev[k] = v[k] / sl;
}

// Eigen Vector4f dot on x86-64 (SSE packet + horizontal add): (p0 + p2) + (p1 + p3)
inline float dot4(const float a[4], const float b[4]) {
    const float p0 = a[0] * b[0], p1 = a[1] * b[1], p2 = a[2] * b[2], p3 = a[3] * b[3];
    return (p0 + p2) + (p1 + p3);
}

}  // namespace

extern "C" int orc_segment(const float* xyz4, const float* nrm4, int w, int h, int* labels_ccl,
                           int* labels_final, orc_region* regions, int max_regions, int* contour,
                           int contour_cap) {
    const size_t N = size_t(w) * h;
    auto P = [&](size_t i, int k) { return xyz4[4 * i + k]; };
    auto Nr = [&](size_t i, int k) { return nrm4[4 * i + k]; };
    const unsigned min_inliers = 80;
    const float ang_thr = std::cos(float(0.039812));       // setAngularThreshold stores cosf
    const float dist_thr = float(0.02);
    const float max_curvature = 0.001f;                     // OMPS maximum_curvature_ default
    // plane_d[i] = p . n
    std::vector<float> plane_d(N);
    for (size_t i = 0; i < N; ++i) plane_d[i] = P(i, 0) * Nr(i, 0) + P(i, 1) * Nr(i, 1) + P(i, 2) * Nr(i, 2);
    // PlaneCoefficientComparator::compare, depth dependent (threshold * z1^2)
    auto compare = [&](size_t a, size_t b) {
        float thr = dist_thr;
        const float z = P(a, 0) * 0.f + P(a, 1) * 0.f + P(a, 2) * 1.f;
        thr *= z * z;
        const float nd = Nr(a, 0) * Nr(b, 0) + Nr(a, 1) * Nr(b, 1) + Nr(a, 2) * Nr(b, 2);
        return std::fabs(plane_d[a] - plane_d[b]) < thr && nd > ang_thr;
    };
    // OrganizedConnectedComponentSegmentation::segment
    const unsigned INV = std::numeric_limits<unsigned>::max();
    std::vector<unsigned> lab(N, INV), run_ids;
    unsigned clust_id = 0;
    auto findRoot = [&](unsigned i) { while (run_ids[i] != i) i = run_ids[i]; return i; };
    auto newRun = [&](size_t i) { lab[i] = clust_id++; run_ids.push_back(lab[i]); };
    if (isfin(P(0, 0))) newRun(0);
    for (int c = 1; c < w; ++c) {
        if (!isfin(P(c, 0))) continue;
        if (compare(c, c - 1)) lab[c] = lab[c - 1];
        else newRun(c);
    }
    for (int r = 1; r < h; ++r) {
        const size_t cur = size_t(r) * w, prev = cur - w;
        if (isfin(P(cur, 0))) {
            if (compare(cur, prev)) lab[cur] = lab[prev];
            else newRun(cur);
        }
        for (int c = 1; c < w; ++c) {
            const size_t i = cur + c;
            if (!isfin(P(i, 0))) continue;
            if (compare(i, i - 1)) lab[i] = lab[i - 1];
            if (compare(i, prev + c)) {
                if (lab[i] == INV) lab[i] = lab[prev + c];
                else if (lab[prev + c] != INV) {
                    const unsigned r1 = findRoot(lab[i]), r2 = findRoot(lab[prev + c]);
                    if (r1 < r2) run_ids[r2] = r1;
                    else run_ids[r1] = r2;
                }
            }
            if (lab[i] == INV) newRun(i);
        }
    }
    std::vector<unsigned> map(clust_id);
    unsigned max_id = 0;
    for (unsigned k = 0; k < run_ids.size(); ++k) map[k] = run_ids[k] == k ? max_id++ : map[findRoot(k)];
    std::vector<std::vector<int>> label_indices(max_id + 1);
    for (size_t i = 0; i < N; ++i)
        if (lab[i] != INV) {
            lab[i] = map[lab[i]];
            label_indices[lab[i]].push_back(int(i));
        }
    for (size_t i = 0; i < N; ++i) labels_ccl[i] = lab[i] == INV ? -1 : int(lab[i]);

    // OrganizedMultiPlaneSegmentation::segment: fit planes to labels with > min_inliers points
    struct Model { float v[4]; float centroid[4]; float cov[9]; float curv; int label; };
    std::vector<Model> models;
    std::vector<std::vector<int>> inliers;
    float vp[4] = {0, 0, 0, 0};
    for (size_t l = 0; l < label_indices.size(); ++l) {
        if (!(unsigned(label_indices[l].size()) > min_inliers)) continue;
        orc_moments::Moments mo;
        for (int i : label_indices[l])
            if (isfin(P(i, 0)) && isfin(P(i, 1)) && isfin(P(i, 2))) mo.add(P(i, 0), P(i, 1), P(i, 2));
        double mean[3], cv[9];
        mo.mean_cov(mean, cv);
        Model m;
        for (int k = 0; k < 3; ++k) m.centroid[k] = float(mean[k]);
        m.centroid[3] = 1;
        for (int k = 0; k < 9; ++k) m.cov[k] = float(cv[k]);
        float eval, evec[3];
        eigen33_min(m.cov, eval, evec);
        float pp[4] = {evec[0], evec[1], evec[2], 0};
        pp[3] = -1 * dot4(pp, m.centroid);
        for (int k = 0; k < 4; ++k) vp[k] -= m.centroid[k];            // accumulates across labels
        const float cos_theta = dot4(vp, pp);
        if (cos_theta < 0) {
            for (int k = 0; k < 4; ++k) pp[k] *= -1;
            pp[3] = -1 * dot4(pp, m.centroid);
        }
        const float eig_sum = m.cov[0] + m.cov[4] + m.cov[8];
        m.curv = eig_sum != 0 ? std::fabs(eval / eig_sum) : 0.f;
        if (m.curv < max_curvature) {
            for (int k = 0; k < 4; ++k) m.v[k] = pp[k];
            m.label = int(l);
            models.push_back(m);
            inliers.push_back(label_indices[l]);
        }
    }

    // refine(): grow the planar labels into neighbouring labelled pixels
    std::vector<char> grow(label_indices.size(), 0);
    std::vector<int> label_to_model(label_indices.size(), 0);
    for (size_t i = 0; i < models.size(); ++i) {
        const int ml = int(lab[inliers[i][0]]);
        label_to_model[ml] = int(i);
        grow[ml] = 1;
    }
    std::vector<int> L(N);
    for (size_t i = 0; i < N; ++i) L[i] = labels_ccl[i];
    auto rcompare = [&](size_t a, size_t b) {                     // PlaneRefinementComparator
        const int cl = L[a], nl = L[b];
        if (!(grow[cl] && !grow[nl])) return false;
        const float* mc = models[label_to_model[cl]].v;
        const double ptp = std::fabs(mc[0] * P(b, 0) + mc[1] * P(b, 1) + mc[2] * P(b, 2) + mc[3]);
        return ptp < dist_thr;
    };
    for (int r = 0; r < h - 1; ++r) {
        const size_t cur = size_t(r) * w, next = cur + w;
        for (int c = 0; c < w - 1; ++c) {
            const int cl = L[cur + c], rl = L[cur + c + 1];
            if (cl < 0 || rl < 0) continue;
            if (rcompare(cur + c, cur + c + 1)) {
                L[cur + c + 1] = cl;
                inliers[label_to_model[cl]].push_back(int(cur + c + 1));
            }
            const int dl = L[next + c];
            if (dl < 0) continue;
            if (rcompare(cur + c, next + c)) {
                L[next + c] = cl;
                inliers[label_to_model[cl]].push_back(int(next + c));
            }
        }
    }
    for (int r = h - 1; r >= 1; --r) {
        const size_t cur = size_t(r) * w, prev = cur - w;
        for (int c = w - 1; c >= 0; --c) {
            const int cl = L[cur + c], ll = L[cur + c - 1];          // c == 0 reads the previous row's end
            if (cl < 0 || ll < 0) continue;
            if (rcompare(cur + c, cur + c - 1)) {
                L[cur + c - 1] = cl;
                inliers[label_to_model[cl]].push_back(int(cur + c - 1));
            }
            const int ul = L[prev + c];
            if (ul < 0) continue;
            if (rcompare(cur + c, prev + c)) {
                L[prev + c] = cl;
                inliers[label_to_model[cl]].push_back(int(prev + c));
            }
        }
    }
    for (size_t i = 0; i < N; ++i) labels_final[i] = L[i];

    // boundaries: OrganizedConnectedComponentSegmentation::findLabeledRegionBoundary
    if (int(models.size()) > max_regions) return -1;
    const int dxs[8] = {-1, -1, 0, 1, 1, 1, 0, -1}, dys[8] = {0, -1, -1, -1, 0, 1, 1, 1};
    int coff = 0;
    for (size_t m = 0; m < models.size(); ++m) {
        orc_region& R = regions[m];
        const int start = inliers[m][0];
        R.label = models[m].label;
        R.count = int(inliers[m].size());
        R.start_idx = start;
        for (int k = 0; k < 3; ++k) R.centroid[k] = models[m].centroid[k];
        for (int k = 0; k < 9; ++k) R.cov[k] = models[m].cov[k];
        for (int k = 0; k < 4; ++k) R.model[k] = models[m].v[k];
        R.curvature = models[m].curv;
        R.contour_off = coff;
        R.n_contour = 0;
        const int label = L[start];
        int cx = start % w, cy = start / w, cidx = start, dir = -1;
        for (int d = 0; d < 8; ++d) {
            const int x = cx + dxs[d], y = cy + dys[d];
            if (x >= 0 && x < w && y >= 0 && y < h && L[cidx + dys[d] * w + dxs[d]] != label) { dir = d; break; }
        }
        if (dir < 0) continue;
        if (coff >= contour_cap) return -1;
        contour[coff++] = start;
        do {
            int nd = 0;
            for (int d = 1; d <= 8; ++d) {
                nd = (dir + d) & 7;
                const int x = cx + dxs[nd], y = cy + dys[nd];
                if (x >= 0 && x < w && y >= 0 && y < h && L[cidx + dys[nd] * w + dxs[nd]] == label) break;
            }
            dir = (nd + 4) & 7;
            cidx += dys[nd] * w + dxs[nd];
            cx += dxs[nd];
            cy += dys[nd];
            if (coff >= contour_cap) return -1;
            contour[coff++] = cidx;
        } while (cidx != start);
        R.n_contour = coff - R.contour_off;
    }
    return int(models.size());
}
