// photo_icp_oracle.cpp — ORACLE (test infrastructure only, see oracle360.h).
// Restatement of RegisterPhotoICP's spherical dense registration path
// (include/RegisterPhotoICP.h).  Per-pixel arithmetic follows the reference's
// float/double mix expression by expression; the image-wide sums are taken in
// double (the reference's OpenMP float reduction is thread-count dependent,
// :3117-3195, so the double sum is the value it approximates).
#include "oracle360.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

static const double REF_PI = 3.14159265359;          // include/Miscellaneous.h:44
static const float INVALID_POINT = -10000;           // include/RegisterPhotoICP.h:40

// ---------------------------------------------------------------------------
// A14 pre-processing
// ---------------------------------------------------------------------------
// cv::cvtColor(imgRGB, gray, CV_RGB2GRAY) on BGR-stored data (:485, :502): OpenCV 8-bit
// fixed point (yuv_shift 14; R2Y 4899, G2Y 9617, B2Y 1868), channel 0 weighted as R.
// Then convertTo(CV_32FC1, 1./255): float scale (cvtScale_<uchar,float,float>).
extern "C" void orc_rgb2gray(const uint8_t* bgr, int n, float* gray) {
    const float scale = (float)(1. / 255);
    for (int i = 0; i < n; ++i) {
        int y = (bgr[3 * i] * 4899 + bgr[3 * i + 1] * 9617 + bgr[3 * i + 2] * 1868 + (1 << 13)) >> 14;
        gray[i] = (float)y * scale;
    }
}

// buildPyramidRange level 0: CV_16U -> convertTo(CV_32FC1, 0.001) (:316-317)
extern "C" void orc_depth_to_m(const uint16_t* d, int n, float* out) {
    const float scale = (float)0.001;
    for (int i = 0; i < n; ++i) out[i] = (float)d[i] * scale;
}

static inline int reflect101(int p, int n) {  // cv::BORDER_REFLECT_101
    if (n == 1) return 0;
    while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - p - 2;
    return p;
}

// cv::pyrDown(src, dst, Size(cols/2, rows/2)) for CV_32F (buildPyramid :292-308):
// horizontal [1 4 6 4 1] decimation in float (scalar order of pyrDown_), vertical pass
// in the SSE order of PyrDownVec_32f, times 1/256.  Border: BORDER_REFLECT_101.
extern "C" void orc_pyrdown(const float* src, int rows, int cols, float* dst) {
    const int dr = rows / 2, dc = cols / 2;
    std::vector<float> hrow((size_t)rows * dc);
    for (int y = 0; y < rows; ++y) {
        const float* s = src + (size_t)y * cols;
        for (int x = 0; x < dc; ++x) {
            int sx = 2 * x;
            float a = s[reflect101(sx - 2, cols)], b = s[reflect101(sx - 1, cols)], c = s[sx],
                  d = s[reflect101(sx + 1, cols)], e = s[reflect101(sx + 2, cols)];
            hrow[(size_t)y * dc + x] = c * 6 + (b + d) * 4 + a + e;
        }
    }
    const float scale = 1.f / 256;
    for (int y = 0; y < dr; ++y) {
        const float* r0 = &hrow[(size_t)reflect101(2 * y - 2, rows) * dc];
        const float* r1 = &hrow[(size_t)reflect101(2 * y - 1, rows) * dc];
        const float* r2 = &hrow[(size_t)(2 * y) * dc];
        const float* r3 = &hrow[(size_t)reflect101(2 * y + 1, rows) * dc];
        const float* r4 = &hrow[(size_t)reflect101(2 * y + 2, rows) * dc];
        for (int x = 0; x < dc; ++x) {
            float t0 = r0[x] + r4[x];
            float t1 = (r1[x] + r3[x]) + r2[x];
            t0 = t0 + (r2[x] + r2[x]);
            t0 = t0 + t1 * 4.f;
            dst[(size_t)y * dc + x] = t0 * scale;
        }
    }
}

// buildPyramidRange (:312-354): 2x2 mean of the depths in (minDepth, maxDepth), else 0.
extern "C" void orc_pyr_range(const float* src, int rows, int cols, float min_d, float max_d, float* dst) {
    const int dc = cols / 2;
    for (int r = 0; r < rows; r += 2)
        for (int c = 0; c < cols; c += 2) {
            float av = 0.f; unsigned nv = 0;
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) {
                    float z = src[(size_t)(r + i) * cols + c + j];
                    if (z > min_d && z < max_d) { av += z; ++nv; }
                }
            dst[(size_t)(r / 2) * dc + c / 2] = nv > 0 ? av / nv : 0.f;
        }
}

// calcGradientXY (:365-398): harmonic-mean derivative where the signal is strictly monotone.
extern "C" void orc_gradient(const float* s, int rows, int cols, float* gx, float* gy) {
    memset(gx, 0, sizeof(float) * rows * cols);
    memset(gy, 0, sizeof(float) * rows * cols);
    for (int r = 1; r < rows - 1; ++r)
        for (int c = 1; c < cols - 1; ++c) {
            size_t i = (size_t)r * cols + c;
            float f = s[i], fr = s[i + 1], fl = s[i - 1], fd = s[i + cols], fu = s[i - cols];
            if ((f > fr && f < fl) || (f < fr && f > fl))
                gx[i] = 2.f / (1 / (fr - f) + 1 / (f - fl));
            if ((f > fd && f < fu) || (f < fd && f > fu))
                gy[i] = 2.f / (1 / (fd - f) + 1 / (f - fu));
        }
}

extern "C" float orc_huber(float e, float reg) {               // :545-554 (T = float)
    float a = std::fabs(e);
    if (a < reg) return 1.f;
    return std::sqrt(2 * reg * a - reg * reg) / a;
}

// ---------------------------------------------------------------------------
// Sphere LUT (alignFrames360 :4553-4587)
// ---------------------------------------------------------------------------
struct Lut { std::vector<float> x, y, z; };

static void build_lut(const orc_level* L, float min_d, float max_d, Lut& lut) {
    const int R = L->rows, C = L->cols;
    lut.x.resize((size_t)R * C); lut.y.resize((size_t)R * C); lut.z.resize((size_t)R * C);
    const float angle_res = 2 * REF_PI / C;
    std::vector<float> st(C), ct(C);
    for (int c = 0; c < C; ++c) { float th = c * angle_res; st[c] = std::sin(th); ct[c] = std::cos(th); }
    const float half_nRows = 0.5 * R - 0.5;
    for (int r = 0; r < R; ++r) {
        float phi = (half_nRows - r) * angle_res;
        float sp = std::sin(phi), cp = std::cos(phi);
        for (int c = 0; c < C; ++c) {
            size_t i = (size_t)r * C + c;
            float d = L->depth_src[i];
            if (min_d < d && d < max_d) {
                lut.x[i] = d * sp;
                lut.y[i] = -d * cp * st[c];
                lut.z[i] = -d * cp * ct[c];
            } else {
                lut.x[i] = INVALID_POINT;
            }
        }
    }
}

struct Pose { float R[9]; float t[3]; };  // R row-major
static Pose split_pose(const float T[16]) {
    Pose p;
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) p.R[r * 3 + c] = T[c * 4 + r];
        p.t[r] = T[12 + r];
    }
    return p;
}

// Transform + spherical projection shared by :2672-2684 and :2973-2989.
struct Proj { float x, y, z, dist, dist_inv; int r, c; bool vis; };
static inline Proj project(const Pose& P, float lx, float ly, float lz, int nRows, int nCols,
                           float half_nRows, float angle_res_inv) {
    Proj o;
    // Eigen: rotation*p + translation
    o.x = P.R[0] * lx + P.R[1] * ly + P.R[2] * lz; o.x = o.x + P.t[0];
    o.y = P.R[3] * lx + P.R[4] * ly + P.R[5] * lz; o.y = o.y + P.t[1];
    o.z = P.R[6] * lx + P.R[7] * ly + P.R[8] * lz; o.z = o.z + P.t[2];
    o.dist = std::sqrt(o.x * o.x + o.y * o.y + o.z * o.z);
    o.dist_inv = 1.f / o.dist;
    float phi_trg = std::asin(o.x * o.dist_inv);
    float theta_trg = (float)(std::atan2(o.y, o.z) + REF_PI);
    o.r = (int)std::round(half_nRows - phi_trg * angle_res_inv);
    o.c = (int)std::round(theta_trg * angle_res_inv);
    o.vis = (o.r >= 0 && o.r < nRows) && o.c < nCols;
    return o;
}

// ---------------------------------------------------------------------------
// A16 — errorPhotoICP_sphere (:2545-2739)
// ---------------------------------------------------------------------------
static double error_sphere_lut(const orc_level* L, const Lut& lut, const float pose[16], int method,
                               const orc_icp_params* p, int* n_valid, double* err2_out) {
    const int nRows = L->rows, nCols = L->cols;
    const float angle_res = 2 * REF_PI / nCols;
    const float angle_res_inv = 1 / angle_res;
    const float half_nRows = 0.5 * nRows - 0.5;
    const double stdDevPhoto_inv = 1. / p->std_dev_photo;
    const Pose P = split_pose(pose);
    const long N = (long)nRows * nCols;
    double error2 = 0.0; long nv = 0;
    #pragma omp parallel for reduction(+ : error2, nv) schedule(static)
    for (long i = 0; i < N; ++i) {
        if (lut.x[i] == INVALID_POINT) continue;
        Proj o = project(P, lut.x[i], lut.y[i], lut.z[i], nRows, nCols, half_nRows, angle_res_inv);
        if (!o.vis) continue;
        size_t t = (size_t)o.r * nCols + o.c;
        if (method == ORC_PHOTO || method == ORC_PHOTO_DEPTH) {
            if (std::fabs(L->gx[t]) < p->thres_sal_int && std::fabs(L->gy[t]) < p->thres_sal_int) continue;
            float photoDiff = L->gray_trg[t] - L->gray_src[i];
            double weight_photo = orc_huber(photoDiff, p->std_dev_photo) * stdDevPhoto_inv;
            float wE = (float)(weight_photo * photoDiff);
            error2 += wE * wE;
            ++nv;
        }
        if (method == ORC_DEPTH || method == ORC_PHOTO_DEPTH) {
            float depth2 = L->depth_trg[t];
            if (std::isfinite(depth2)) {
                if (std::fabs(L->dgx[t]) < p->thres_sal_depth && std::fabs(L->dgy[t]) < p->thres_sal_depth) continue;
                float depthDiff = depth2 - o.dist;
                float sd = p->std_dev_depth * depth2;
                double weight_depth = orc_huber(depthDiff, sd) / sd;
                float wE = (float)(weight_depth * depthDiff);
                error2 += wE * wE;
                ++nv;
            }
        }
    }
    *n_valid = (int)nv;
    if (err2_out) *err2_out = error2;
    return std::sqrt(error2 / nv);
}

// ---------------------------------------------------------------------------
// A17 — calcHessGrad_sphere (:2745-3228)
// ---------------------------------------------------------------------------
static void hessgrad_sphere_lut(const orc_level* L, const Lut& lut, const float pose[16], int method,
                                const orc_icp_params* p, double H[36], double g[6], int* n_visible) {
    const int nRows = L->rows, nCols = L->cols;
    const float angle_res = 2 * REF_PI / nCols;
    const float angle_res_inv = 1 / angle_res;
    const float half_nRows = 0.5 * nRows - 0.5;
    const float stdDevPhoto_inv = 1. / p->std_dev_photo;
    const Pose P = split_pose(pose);
    const long N = (long)nRows * nCols;
    double acc[27] = {0};
    long nvis = 0;
    #pragma omp parallel
    {
        double a[27] = {0};
        long lv = 0;
        #pragma omp for schedule(static)
        for (long i = 0; i < N; ++i) {
            if (lut.x[i] == INVALID_POINT) continue;
            Proj o = project(P, lut.x[i], lut.y[i], lut.z[i], nRows, nCols, half_nRows, angle_res_inv);
            if (!o.vis) continue;
            ++lv;
            const float X = o.x, Y = o.y, Z = o.z;
            // jacobianT36 = [I | -skew(p')]  (:2995-2997; skew: include/Miscellaneous.h:87-98)
            float T[3][6] = {{1, 0, 0, 0, Z, -Y}, {0, 1, 0, -Z, 0, X}, {0, 0, 1, Y, -X, 0}};
            // jacobianProj23 (:3000-3016)
            float z_inv = 1.f / Z;
            float z_inv2 = z_inv * z_inv;
            float D_atan_theta = 1.f / (1 + Y * Y * z_inv2) * angle_res_inv;
            float Pj[2][3];
            Pj[0][0] = 0;
            Pj[0][1] = D_atan_theta * z_inv;
            Pj[0][2] = -Y * z_inv2 * D_atan_theta;
            float dist_inv2 = o.dist_inv * o.dist_inv;
            float x_dist_inv2 = X * dist_inv2;
            float D_asin = 1.f / std::sqrt(1 - X * x_dist_inv2) * angle_res_inv;
            Pj[1][0] = -D_asin * o.dist_inv * (1 - X * x_dist_inv2);
            Pj[1][1] = D_asin * (x_dist_inv2 * Y * o.dist_inv);
            Pj[1][2] = D_asin * (x_dist_inv2 * Z * o.dist_inv);
            float Jw[2][6];  // jacobianWarpRt = jacobianProj23 * jacobianT36 (:3026)
            for (int r = 0; r < 2; ++r)
                for (int c = 0; c < 6; ++c) Jw[r][c] = Pj[r][0] * T[0][c] + Pj[r][1] * T[1][c] + Pj[r][2] * T[2][c];
            size_t t = (size_t)o.r * nCols + o.c;
            if (method == ORC_PHOTO || method == ORC_PHOTO_DEPTH) {
                float gx = L->gx[t], gy = L->gy[t];
                if (std::fabs(gx) < p->thres_sal_int && std::fabs(gy) < p->thres_sal_int) continue;  // :3038-3039
                float photoDiff = L->gray_trg[t] - L->gray_src[i];
                float weight_photo = orc_huber(photoDiff, p->std_dev_photo) * stdDevPhoto_inv;
                float r = weight_photo * photoDiff;
                float J[6];
                // (weight_photo * target_imgGradient) * jacobianWarpRt  (:3052, left-to-right)
                const float wgx = weight_photo * gx, wgy = weight_photo * gy;
                for (int c = 0; c < 6; ++c) J[c] = wgx * Jw[0][c] + wgy * Jw[1][c];
                int k = 0;
                for (int u = 0; u < 6; ++u)
                    for (int v = u; v < 6; ++v) a[k++] += (double)(J[u] * J[v]);
                for (int u = 0; u < 6; ++u) a[21 + u] += (double)(J[u] * r);
            }
            if (method == ORC_DEPTH || method == ORC_PHOTO_DEPTH) {
                float depth2 = L->depth_trg[t];
                if (std::isfinite(depth2)) {
                    float dgx = L->dgx[t], dgy = L->dgy[t];
                    if (std::fabs(dgx) < p->thres_sal_depth && std::fabs(dgy) < p->thres_sal_depth) continue;
                    float depthDiff = depth2 - o.dist;
                    float sd = p->std_dev_depth * depth2;
                    float weight_depth = orc_huber(depthDiff, sd) / sd;
                    float r = weight_depth * depthDiff;
                    float js0 = X * o.dist_inv, js1 = Y * o.dist_inv, js2 = Z * o.dist_inv;
                    float J[6];
                    for (int c = 0; c < 6; ++c) {
                        float ga = dgx * Jw[0][c] + dgy * Jw[1][c];
                        float gb = js0 * T[0][c] + js1 * T[1][c] + js2 * T[2][c];
                        J[c] = weight_depth * (ga - gb);
                    }
                    int k = 0;
                    for (int u = 0; u < 6; ++u)
                        for (int v = u; v < 6; ++v) a[k++] += (double)(J[u] * J[v]);
                    for (int u = 0; u < 6; ++u) a[21 + u] += (double)(J[u] * r);
                }
            }
        }
        #pragma omp critical
        {
            for (int k = 0; k < 27; ++k) acc[k] += a[k];
            nvis += lv;
        }
    }
    int k = 0;
    for (int u = 0; u < 6; ++u)
        for (int v = u; v < 6; ++v) { H[u * 6 + v] = H[v * 6 + u] = acc[k++]; }
    for (int u = 0; u < 6; ++u) g[u] = acc[21 + u];
    *n_visible = (int)nvis;
}

// ---------------------------------------------------------------------------
// §8(f)1 — occlusion-aware variants (alignFrames360 occlusion = 1 / 2, :4598-4627).  The reference
// runs these loops under `omp parallel for` with unsynchronised Z-buffer and residual writes (a data
// race); the restatement takes the single-thread order, LUT index i ascending, which is the only
// deterministic reading.
// ---------------------------------------------------------------------------
static const float kThresDepthOutliers = 0.3f;   // alignFrames360 :4525
// the members errorPhotoICP_sphereOcc1/2 assign (avPhotoResidual / avDepthResidual, :3360-3362, :3852-3853)
static thread_local double g_avPhoto = 0.0, g_avDepth = 0.0;

// errorPhotoICP_sphereOcc1 (:3232-3370): Z-buffer on the TARGET pixel; an accepted point overwrites
// the pixel's residual, every accepted point counts.  Returns avPhotoResidual + avDepthResidual.
static double error_sphere_occ1(const orc_level* L, const Lut& lut, const float pose[16], int method,
                                const orc_icp_params* p, int* n_valid) {
    const int nRows = L->rows, nCols = L->cols;
    const float angle_res = 2 * REF_PI / nCols;
    const float angle_res_inv = 1 / angle_res;
    const float half_nRows = 0.5 * nRows - 0.5;
    const double stdDevPhoto_inv = 1. / p->std_dev_photo;
    const Pose P = split_pose(pose);
    const long N = (long)nRows * nCols;
    std::vector<float> zbuf(N, 0.f), resP(N, 0.f), resD(N, 0.f);
    long nP = 0, nD = 0;
    for (long i = 0; i < N; ++i) {
        if (lut.x[i] == INVALID_POINT) continue;
        Proj o = project(P, lut.x[i], lut.y[i], lut.z[i], nRows, nCols, half_nRows, angle_res_inv);
        if (!o.vis) continue;
        const size_t ii = (size_t)o.r * nCols + o.c;
        if (zbuf[ii] > 0 && o.dist_inv < zbuf[ii]) continue;      // occluded (:3292-3294)
        zbuf[ii] = o.dist_inv;
        if (method == ORC_PHOTO || method == ORC_PHOTO_DEPTH) {
            if (std::fabs(L->gx[ii]) < p->thres_sal_int && std::fabs(L->gy[ii]) < p->thres_sal_int) continue;
            float photoDiff = L->gray_trg[ii] - L->gray_src[i];
            double weight_photo = orc_huber(photoDiff, p->std_dev_photo) * stdDevPhoto_inv;
            float wE = (float)(weight_photo * photoDiff);
            resP[ii] = wE * wE;
            ++nP;
        }
        if (method == ORC_DEPTH || method == ORC_PHOTO_DEPTH) {
            float depth2 = L->depth_trg[ii];
            if (std::isfinite(depth2)) {
                if (std::fabs(L->dgx[ii]) < p->thres_sal_depth && std::fabs(L->dgy[ii]) < p->thres_sal_depth) continue;
                float depthDiff = depth2 - o.dist;
                float sd = p->std_dev_depth * depth2;
                double weight_depth = orc_huber(depthDiff, sd) / sd;
                float wE = (float)(weight_depth * depthDiff);
                resD[ii] = wE * wE;
                ++nD;
            }
        }
    }
    double PR = 0.0, DR = 0.0;
    for (long i = 0; i < N; ++i) { PR += resP[i]; DR += resD[i]; }
    *n_valid = (int)(nP + nD);
    g_avPhoto = std::sqrt(PR / nP);
    g_avDepth = std::sqrt(DR / nD);
    return g_avPhoto + g_avDepth;
}

// errorPhotoICP_sphereOcc2 (:3720-3855): depth-outlier filter, then the target Z-buffer; residuals are
// kept per SOURCE point, so every accepted point contributes.  Both averages use nValidDepthPts.
static double error_sphere_occ2(const orc_level* L, const Lut& lut, const float pose[16], int method,
                                const orc_icp_params* p, int* n_valid) {
    const int nRows = L->rows, nCols = L->cols;
    const float angle_res = 2 * REF_PI / nCols;
    const float angle_res_inv = 1 / angle_res;
    const float half_nRows = 0.5 * nRows - 0.5;
    const double stdDevPhoto_inv = 1. / p->std_dev_photo;
    const Pose P = split_pose(pose);
    const long N = (long)nRows * nCols;
    std::vector<float> zbuf(N, 0.f), resP(N, 0.f), resD(N, 0.f);
    long nV = 0;
    for (long i = 0; i < N; ++i) {
        if (lut.x[i] == INVALID_POINT) continue;
        Proj o = project(P, lut.x[i], lut.y[i], lut.z[i], nRows, nCols, half_nRows, angle_res_inv);
        if (!o.vis) continue;
        const size_t ii = (size_t)o.r * nCols + o.c;
        float depth2 = L->depth_trg[ii];
        float depthDiff = depth2 - o.dist;
        if (std::fabs(depthDiff) > kThresDepthOutliers) continue;     // :3790-3791
        if (zbuf[ii] > 0 && o.dist_inv < zbuf[ii]) continue;         // :3794-3796
        zbuf[ii] = o.dist_inv;
        ++nV;
        if (method == ORC_PHOTO || method == ORC_PHOTO_DEPTH) {
            if (std::fabs(L->gx[ii]) < p->thres_sal_int && std::fabs(L->gy[ii]) < p->thres_sal_int) continue;
            float photoDiff = L->gray_trg[ii] - L->gray_src[i];
            double weight_photo = orc_huber(photoDiff, p->std_dev_photo) * stdDevPhoto_inv;
            float wE = (float)(weight_photo * photoDiff);
            resP[i] = wE * wE;
        }
        if (method == ORC_DEPTH || method == ORC_PHOTO_DEPTH) {
            if (std::isfinite(depth2)) {
                if (std::fabs(L->dgx[ii]) < p->thres_sal_depth && std::fabs(L->dgy[ii]) < p->thres_sal_depth) continue;
                float sd = p->std_dev_depth * depth2;
                double weight_depth = orc_huber(depthDiff, sd) / sd;
                float wE = (float)(weight_depth * depthDiff);
                resD[i] = wE * wE;
            }
        }
    }
    double PR = 0.0, DR = 0.0;
    for (long i = 0; i < N; ++i) { PR += resP[i]; DR += resD[i]; }
    *n_valid = (int)nV;
    g_avPhoto = std::sqrt(PR / nV);
    g_avDepth = std::sqrt(DR / nV);
    return g_avPhoto + g_avDepth;
}

// calcHessGrad_sphereOcc2 (:3861-4250): depth-outlier filter; the LAST filtered point of each target
// pixel (LUT order) owns that pixel's Jacobian rows and residuals.  A depth-saliency `continue` skips
// the store of both rows.  numVisiblePixels counts target pixels hit by a filtered point.
// (calcHessGrad_sphereOcc1 indexes its Z-buffer by the source index, :3486-3488, so it never occludes
// and equals calcHessGrad_sphere.)
static void hessgrad_sphere_occ2(const orc_level* L, const Lut& lut, const float pose[16], int method,
                                 const orc_icp_params* p, double H[36], double g[6], int* n_visible) {
    const int nRows = L->rows, nCols = L->cols;
    const float angle_res = 2 * REF_PI / nCols;
    const float angle_res_inv = 1 / angle_res;
    const float half_nRows = 0.5 * nRows - 0.5;
    const float stdDevPhoto_inv = 1. / p->std_dev_photo;
    const Pose P = split_pose(pose);
    const long N = (long)nRows * nCols;
    std::vector<float> zbuf(N, 0.f), JP(6 * N), JD(6 * N), rP(N), rD(N);
    std::vector<char> vP(N, 0), vD(N, 0);
    long nvis = 0;
    for (long i = 0; i < N; ++i) {
        if (lut.x[i] == INVALID_POINT) continue;
        Proj o = project(P, lut.x[i], lut.y[i], lut.z[i], nRows, nCols, half_nRows, angle_res_inv);
        if (!o.vis) continue;
        const size_t ii = (size_t)o.r * nCols + o.c;
        float depth2 = L->depth_trg[ii];
        float depthDiff = depth2 - o.dist;
        if (std::fabs(depthDiff) > kThresDepthOutliers) continue;
        if (zbuf[ii] == 0) ++nvis;
        zbuf[ii] = o.dist_inv;
        const float X = o.x, Y = o.y, Z = o.z;
        float T[3][6] = {{1, 0, 0, 0, Z, -Y}, {0, 1, 0, -Z, 0, X}, {0, 0, 1, Y, -X, 0}};
        float z_inv = 1.f / Z;
        float z_inv2 = z_inv * z_inv;
        float D_atan_theta = 1.f / (1 + Y * Y * z_inv2) * angle_res_inv;
        float Pj[2][3];
        Pj[0][0] = 0;
        Pj[0][1] = D_atan_theta * z_inv;
        Pj[0][2] = -Y * z_inv2 * D_atan_theta;
        float dist_inv2 = o.dist_inv * o.dist_inv;
        float x_dist_inv2 = X * dist_inv2;
        float D_asin = 1.f / std::sqrt(1 - X * x_dist_inv2) * angle_res_inv;
        Pj[1][0] = -D_asin * o.dist_inv * (1 - X * x_dist_inv2);
        Pj[1][1] = D_asin * (x_dist_inv2 * Y * o.dist_inv);
        Pj[1][2] = D_asin * (x_dist_inv2 * Z * o.dist_inv);
        float Jw[2][6];
        for (int r = 0; r < 2; ++r)
            for (int c = 0; c < 6; ++c) Jw[r][c] = Pj[r][0] * T[0][c] + Pj[r][1] * T[1][c] + Pj[r][2] * T[2][c];
        float Jp[6] = {0}, Jd[6] = {0}, wEP = 0, wED = 0;
        if (method == ORC_PHOTO || method == ORC_PHOTO_DEPTH) {
            float gx = L->gx[ii], gy = L->gy[ii];
            if (std::fabs(gx) < p->thres_sal_int && std::fabs(gy) < p->thres_sal_int) continue;
            float photoDiff = L->gray_trg[ii] - L->gray_src[i];
            float weight_photo = orc_huber(photoDiff, p->std_dev_photo) * stdDevPhoto_inv;
            wEP = weight_photo * photoDiff;
            const float wgx = weight_photo * gx, wgy = weight_photo * gy;
            for (int c = 0; c < 6; ++c) Jp[c] = wgx * Jw[0][c] + wgy * Jw[1][c];
        }
        if (method == ORC_DEPTH || method == ORC_PHOTO_DEPTH) {
            if (std::isfinite(depth2)) {
                float dgx = L->dgx[ii], dgy = L->dgy[ii];
                if (std::fabs(dgx) < p->thres_sal_depth && std::fabs(dgy) < p->thres_sal_depth) continue;
                float sd = p->std_dev_depth * depth2;
                float weight_depth = orc_huber(depthDiff, sd) / sd;
                wED = weight_depth * depthDiff;
                float js0 = X * o.dist_inv, js1 = Y * o.dist_inv, js2 = Z * o.dist_inv;
                for (int c = 0; c < 6; ++c) {
                    float ga = dgx * Jw[0][c] + dgy * Jw[1][c];
                    float gb = js0 * T[0][c] + js1 * T[1][c] + js2 * T[2][c];
                    Jd[c] = weight_depth * (ga - gb);
                }
            }
        }
        if (method == ORC_PHOTO || method == ORC_PHOTO_DEPTH) {
            for (int c = 0; c < 6; ++c) JP[6 * ii + c] = Jp[c];
            rP[ii] = wEP;
            vP[ii] = 1;
        }
        if ((method == ORC_DEPTH || method == ORC_PHOTO_DEPTH) && std::isfinite(depth2)) {
            for (int c = 0; c < 6; ++c) JD[6 * ii + c] = Jd[c];
            rD[ii] = wED;
            vD[ii] = 1;
        }
    }
    double acc[27] = {0};
    for (int pass = 0; pass < 2; ++pass) {
        const std::vector<float>& J = pass ? JD : JP;
        const std::vector<float>& rr = pass ? rD : rP;
        const std::vector<char>& v = pass ? vD : vP;
        for (long i = 0; i < N; ++i) {
            if (!v[i]) continue;
            const float* j = &J[6 * i];
            int k = 0;
            for (int u = 0; u < 6; ++u)
                for (int w = u; w < 6; ++w) acc[k++] += (double)(j[u] * j[w]);
            for (int u = 0; u < 6; ++u) acc[21 + u] += (double)(j[u] * rr[i]);
        }
    }
    int k = 0;
    for (int u = 0; u < 6; ++u)
        for (int w = u; w < 6; ++w) { H[u * 6 + w] = H[w * 6 + u] = acc[k++]; }
    for (int u = 0; u < 6; ++u) g[u] = acc[21 + u];
    *n_visible = (int)nvis;
}

static double error_any(const orc_level* L, const Lut& lut, const float pose[16], int method, int occ,
                        const orc_icp_params* p, int* nv) {
    if (occ == 1) return error_sphere_occ1(L, lut, pose, method, p, nv);
    if (occ == 2) return error_sphere_occ2(L, lut, pose, method, p, nv);
    return error_sphere_lut(L, lut, pose, method, p, nv, nullptr);
}

static void hessgrad_any(const orc_level* L, const Lut& lut, const float pose[16], int method, int occ,
                         const orc_icp_params* p, double H[36], double g[6], int* nvis) {
    if (occ == 2) hessgrad_sphere_occ2(L, lut, pose, method, p, H, g, nvis);
    else hessgrad_sphere_lut(L, lut, pose, method, p, H, g, nvis);
}

extern "C" double orc_error_sphere_occ(const orc_level* L, const float pose[16], int method, int occ,
                                       const orc_icp_params* p, int* n_valid) {
    Lut lut; build_lut(L, p->min_depth, p->max_depth, lut);
    return error_any(L, lut, pose, method, occ, p, n_valid);
}

extern "C" void orc_hessgrad_sphere_occ(const orc_level* L, const float pose[16], int method, int occ,
                                        const orc_icp_params* p, double H[36], double g[6], int* n_visible) {
    Lut lut; build_lut(L, p->min_depth, p->max_depth, lut);
    hessgrad_any(L, lut, pose, method, occ, p, H, g, n_visible);
}

extern "C" double orc_error_sphere(const orc_level* L, const float pose[16], int method,
                                   const orc_icp_params* p, int* n_valid, double* err2) {
    Lut lut; build_lut(L, p->min_depth, p->max_depth, lut);
    return error_sphere_lut(L, lut, pose, method, p, n_valid, err2);
}

extern "C" void orc_hessgrad_sphere(const orc_level* L, const float pose[16], int method,
                                    const orc_icp_params* p, double H[36], double g[6], int* n_visible) {
    Lut lut; build_lut(L, p->min_depth, p->max_depth, lut);
    hessgrad_sphere_lut(L, lut, pose, method, p, H, g, n_visible);
}

// ---------------------------------------------------------------------------
// A18 — mrpt::poses::CPose3D::exp(mu, pseudo) ; mu = [t ; w]
// ---------------------------------------------------------------------------
extern "C" void orc_exp_se3(const double mu[6], int pseudo, float T[16]) {
    const double wx = mu[3], wy = mu[4], wz = mu[5];
    const double th2 = wx * wx + wy * wy + wz * wz, th = std::sqrt(th2);
    double A, B, C;  // sin(t)/t, (1-cos t)/t^2, (t - sin t)/t^3
    if (th < 1e-6) { A = 1 - th2 / 6; B = 0.5 - th2 / 24; C = 1.0 / 6 - th2 / 120; }
    else { A = std::sin(th) / th; B = (1 - std::cos(th)) / th2; C = (th - std::sin(th)) / (th2 * th); }
    const double W[9] = {0, -wz, wy, wz, 0, -wx, -wy, wx, 0};
    double W2[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0; for (int k = 0; k < 3; ++k) s += W[r * 3 + k] * W[k * 3 + c];
            W2[r * 3 + c] = s;
        }
    double R[9], V[9];
    for (int i = 0; i < 9; ++i) {
        double I = (i % 4 == 0) ? 1.0 : 0.0;
        R[i] = I + A * W[i] + B * W2[i];
        V[i] = I + B * W[i] + C * W2[i];
    }
    double t[3];
    for (int r = 0; r < 3; ++r)
        t[r] = pseudo ? mu[r] : V[r * 3] * mu[0] + V[r * 3 + 1] * mu[1] + V[r * 3 + 2] * mu[2];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) {
            double v;
            if (r < 3 && c < 3) v = R[r * 3 + c];
            else if (r < 3) v = t[r];
            else v = (c == 3) ? 1.0 : 0.0;
            T[c * 4 + r] = (float)v;
        }
}

#include "oracle_la.h"

// ---------------------------------------------------------------------------
// A15 — alignFrames360 (:4519-4784) preceded by setTargetFrame / setSourceFrame (:480-516)
// ---------------------------------------------------------------------------
extern "C" int orc_align360_occ(const uint8_t* trg_bgr, const uint16_t* trg_depth,
                                const uint8_t* src_bgr, const uint16_t* src_depth,
                                int rows, int cols, const float init[16], int method, int occlusion,
                                const orc_icp_params* p, float pose_out[16], float H_out[36],
                                float g_out[6], orc_icp_stats* st) {
    const int nL = p->n_pyr;
    std::vector<int> R(nL), C(nL);
    std::vector<std::vector<float>> gs(nL), ds(nL), gt(nL), dt(nL), gx(nL), gy(nL), dgx(nL), dgy(nL);
    for (int l = 0; l < nL; ++l) {
        R[l] = l ? R[l - 1] / 2 : rows; C[l] = l ? C[l - 1] / 2 : cols;
        size_t n = (size_t)R[l] * C[l];
        gs[l].resize(n); ds[l].resize(n); gt[l].resize(n); dt[l].resize(n);
        gx[l].resize(n); gy[l].resize(n); dgx[l].resize(n); dgy[l].resize(n);
    }
    orc_rgb2gray(src_bgr, rows * cols, gs[0].data());
    orc_rgb2gray(trg_bgr, rows * cols, gt[0].data());
    orc_depth_to_m(src_depth, rows * cols, ds[0].data());
    orc_depth_to_m(trg_depth, rows * cols, dt[0].data());
    for (int l = 1; l < nL; ++l) {
        orc_pyrdown(gs[l - 1].data(), R[l - 1], C[l - 1], gs[l].data());
        orc_pyrdown(gt[l - 1].data(), R[l - 1], C[l - 1], gt[l].data());
        orc_pyr_range(ds[l - 1].data(), R[l - 1], C[l - 1], p->min_depth, p->max_depth, ds[l].data());
        orc_pyr_range(dt[l - 1].data(), R[l - 1], C[l - 1], p->min_depth, p->max_depth, dt[l].data());
    }
    for (int l = 0; l < nL; ++l) {
        orc_gradient(gt[l].data(), R[l], C[l], gx[l].data(), gy[l].data());
        orc_gradient(dt[l].data(), R[l], C[l], dgx[l].data(), dgy[l].data());
    }

    if (st) memset(st, 0, sizeof(*st));
    float pose[16]; memcpy(pose, init, sizeof(pose));
    float Hf[36] = {0}, gf[6] = {0};
    int ret = 0;
    for (int l = nL - 1; l >= 0; --l) {
        const int nRows = R[l], nCols = C[l];
        // seam masking of the target gradients (:4538-4549)
        const int ws = nCols / 8;
        for (int s = 1; s < 8; ++s)
            for (int r = 0; r < nRows; ++r)
                for (int c = s * ws - 1; c <= s * ws; ++c) {
                    size_t i = (size_t)r * nCols + c;
                    gx[l][i] = gy[l][i] = dgx[l][i] = dgy[l][i] = 0.f;
                }
        orc_level L = {nRows, nCols, gs[l].data(), ds[l].data(), gt[l].data(), dt[l].data(),
                       gx[l].data(), gy[l].data(), dgx[l].data(), dgy[l].data()};
        Lut lut; build_lut(&L, p->min_depth, p->max_depth, lut);
        const bool fixed = (l == 0 && p->fixed_iters_level0 > 0);
        int it = 0, nv = 0, evals = 0;
        double lambda = p->lambda;                                        // :4589
        const int maxIters = fixed ? p->fixed_iters_level0 : p->max_iters;
        float upd[6] = {1, 1, 1, 1, 1, 1};
        auto note_residuals = [&]() {
            if (st && occlusion) { st->av_photo_residual = g_avPhoto; st->av_depth_residual = g_avDepth; st->residuals_set |= 1; }
        };
        double error = error_any(&L, lut, pose, method, occlusion, p, &nv);
        note_residuals();
        double diff_error = error;
        int loops = 0;
        auto norm6 = [](const float* u) { float s = 0; for (int k = 0; k < 6; ++k) s += u[k] * u[k]; return std::sqrt(s); };
        while (fixed ? loops < maxIters
                     : (it < maxIters && norm6(upd) > p->tol_update && diff_error > p->tol_residual)) {
            ++loops;
            double H[36], g[6]; int nvis = 0;
            hessgrad_any(&L, lut, pose, method, occlusion, p, H, g, &nvis);
            for (int k = 0; k < 36; ++k) Hf[k] = (float)H[k];
            for (int k = 0; k < 6; ++k) gf[k] = (float)g[k];
            if (st) st->sso = (float)nvis / (nRows * nCols);
            double Hd[36], HL[36], gd[6];
            for (int k = 0; k < 36; ++k) Hd[k] = Hf[k];
            for (int k = 0; k < 6; ++k) gd[k] = gf[k];
            // hessian + lambda * diag(hessian): float matrices, the double lambda enters as a float scalar;
            // lambda = 1 at each level start, divided by step = 5 on every accepted update (:4589-4590, :4718)
            memcpy(HL, Hd, sizeof(HL));
            for (int k = 0; k < 6; ++k) HL[k * 7] = (float)(Hf[k * 7] + (float)lambda * Hf[k * 7]);
            if (rank6(HL) != 6) {                                       // :4682-4690
                memcpy(pose_out, pose, sizeof(float) * 16);
                if (st) { st->illposed = 1; st->av_residual = 0.f; st->residuals_set |= 2; }   // avResidual = 0
                ret = 1;
                goto done;
            }
            double x[6];
            solve6(Hd, gd, x);                                            // :4693
            for (int k = 0; k < 6; ++k) upd[k] = (float)x[k];
            double ud[6]; for (int k = 0; k < 6; ++k) ud[k] = upd[k];
            float E[16], cand[16];
            orc_exp_se3(ud, 1, E);                                        // :4697
            matmul4f(E, pose, cand);
            double new_error = error_any(&L, lut, cand, method, occlusion, p, &nv);
            note_residuals();
            ++evals;
            diff_error = error - new_error;                               // :4711
            if (diff_error > p->tol_residual) {                           // :4715-4722
                lambda /= 5.0;                                            // lambda /= step (:4718)
                memcpy(pose, cand, sizeof(pose));
                error = new_error;
                it = it + 1;
            }
        }
        if (st) { st->iters[l] = it; st->evals[l] = evals; st->error = error; }
    }
    memcpy(pose_out, pose, sizeof(pose));
done:
    if (H_out) memcpy(H_out, Hf, sizeof(Hf));
    if (g_out) memcpy(g_out, gf, sizeof(gf));
    return ret;
}

extern "C" int orc_align360(const uint8_t* trg_bgr, const uint16_t* trg_depth,
                            const uint8_t* src_bgr, const uint16_t* src_depth,
                            int rows, int cols, const float init[16], int method,
                            const orc_icp_params* p, float pose_out[16], float H_out[36],
                            float g_out[6], orc_icp_stats* st) {
    return orc_align360_occ(trg_bgr, trg_depth, src_bgr, src_depth, rows, cols, init, method, 0, p, pose_out,
                            H_out, g_out, st);
}

// (M).rank() of Eigen::Matrix<float,6,6> (row-major M), the ILL-POSED test of alignFrames360 (:4682)
extern "C" int orc_rank6f(const float* M) {
    double Md[36];
    for (int k = 0; k < 36; ++k) Md[k] = M[k];
    return rank6(Md);
}

// x = -H^-1 g by the GN step's Gaussian elimination (:4693), H row-major double; 0 when singular
extern "C" int orc_solve6(const double* H, const double* g, double* x) {
    return solve6(H, g, x) ? 1 : 0;
}

// glibc float asinf / atan2f as the reference calls them (std::asin(float), std::atan2(float, float))
extern "C" void orc_libm(const float* x, const float* y, const float* z, int n, float* as, float* at) {
    for (int i = 0; i < n; ++i) { as[i] = std::asin(x[i]); at[i] = std::atan2(y[i], z[i]); }
}
