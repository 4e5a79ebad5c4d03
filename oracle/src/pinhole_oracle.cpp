// pinhole_oracle.cpp — ORACLE (test infrastructure only, see oracle360.h).
// §8(f) rank 3: RegisterPhotoICP's per-sensor pinhole dense registration —
//   alignFrames          include/RegisterPhotoICP.h:4254-4512
//   errorPhotoICP        :560-761   (the non-salient branch, LUT of :4282-4302)
//   calcHessGrad         :767-1100
// as the Methods harness drives it on one sensor of a Frame360 pair
// (Registration/MethodsRegisterRGBD360.cpp:320-345: setCameraMatrix(f = 525*w/640,
// c = (w/2 - 0.5, h/2 - 0.5)), setTargetFrame / setSourceFrame on the raw RGB + u16 depth images).
// Per-pixel arithmetic follows the reference's float expressions; sums are taken in double (the
// reference accumulates H / g in float under `omp critical`, :1080-1097, in arrival order).
#include "oracle360.h"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "oracle_la.h"

static const float INVALID_POINT = -10000;  // include/RegisterPhotoICP.h:40

namespace {

struct Intr { float fx, fy, ox, oy, inv_fx, inv_fy; };

// scaleFactor = 1.0/pow(2, level); fx = cameraMatrix(0,0)*scaleFactor ... (:4273-4279)
Intr level_intrinsics(const orc_pinhole* K, int level) {
    const float s = (float)(1.0 / std::pow(2, level));
    Intr I;
    I.fx = K->fx * s; I.fy = K->fy * s; I.ox = K->ox * s; I.oy = K->oy * s;
    I.inv_fx = (float)(1. / I.fx); I.inv_fy = (float)(1. / I.fy);
    return I;
}

struct Lut { std::vector<float> x, y, z; };

// LUT_xyz_sphere filled with the pinhole back-projection (:4285-4298)
void build_lut(const orc_level* L, const Intr& I, float min_d, float max_d, Lut& lut) {
    const int R = L->rows, C = L->cols;
    lut.x.assign((size_t)R * C, 0.f); lut.y.assign((size_t)R * C, 0.f); lut.z.assign((size_t)R * C, 0.f);
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < C; ++c) {
            const size_t i = (size_t)r * C + c;
            const float z = L->depth_src[i];
            lut.z[i] = z;
            if (min_d < z && z < max_d) {
                lut.x[i] = (c - I.ox) * z * I.inv_fx;
                lut.y[i] = (r - I.oy) * z * I.inv_fy;
            } else {
                lut.x[i] = INVALID_POINT;
            }
        }
}

struct PP { float X, Y, Z, inv; int r, c; bool vis; };

// rotation*LUT + translation, then the pinhole projection (:700-714)
inline PP project(const float T[16], const Lut& lut, size_t i, const Intr& I, int nRows, int nCols) {
    PP o;
    const float lx = lut.x[i], ly = lut.y[i], lz = lut.z[i];
    o.X = T[0] * lx + T[4] * ly + T[8] * lz; o.X = o.X + T[12];
    o.Y = T[1] * lx + T[5] * ly + T[9] * lz; o.Y = o.Y + T[13];
    o.Z = T[2] * lx + T[6] * ly + T[10] * lz; o.Z = o.Z + T[14];
    o.inv = (float)(1.0 / o.Z);
    const float tc = (o.X * I.fx) * o.inv + I.ox;
    const float tr = (o.Y * I.fy) * o.inv + I.oy;
    const float rr = std::round(tr), cc = std::round(tc);
    // (int)round(.) then the bounds test; the float comparison rejects NaN / out-of-range exactly as
    // the x86 conversion (INT_MIN) does
    o.vis = rr >= 0.f && rr < (float)nRows && cc >= 0.f && cc < (float)nCols;
    o.r = o.vis ? (int)rr : 0;
    o.c = o.vis ? (int)cc : 0;
    return o;
}

// errorPhotoICP (:560-761).  avPhotoResidual divides by the DEPTH count (:760), so PHOTO_CONSISTENCY
// (no depth terms) returns NaN, as the reference does.
double error_pin(const orc_level* L, const Lut& lut, const Intr& I, const float pose[16], int method,
                 const orc_icp_params* p, int* n_photo, int* n_depth, double* res_photo, double* res_depth) {
    const int nRows = L->rows, nCols = L->cols;
    const float stdDevPhoto_inv = 1. / p->std_dev_photo;
    const long N = (long)nRows * nCols;
    double P = 0.0, D = 0.0;
    long nP = 0, nD = 0;
    #pragma omp parallel for reduction(+ : P, D, nP, nD) schedule(static)
    for (long i = 0; i < N; ++i) {
        if (lut.x[i] == INVALID_POINT) continue;
        const PP o = project(pose, lut, i, I, nRows, nCols);
        if (!o.vis) continue;
        const size_t t = (size_t)o.r * nCols + o.c;
        if (method == ORC_PHOTO || method == ORC_PHOTO_DEPTH) {
            const float photoDiff = L->gray_trg[t] - L->gray_src[i];
            const float w = orc_huber(photoDiff, p->std_dev_photo) * stdDevPhoto_inv;
            const float wE = w * photoDiff;
            P += wE * wE;
            ++nP;
        }
        if (method == ORC_DEPTH || method == ORC_PHOTO_DEPTH) {
            const float depth2 = L->depth_trg[t];
            if (std::isfinite(depth2)) {
                const float depthDiff = depth2 - o.Z;
                const float sd = p->std_dev_depth * o.Z;
                const float w = orc_huber(depthDiff, sd) / sd;
                const float wE = w * depthDiff;
                D += wE * wE;
                ++nD;
            }
        }
    }
    if (n_photo) *n_photo = (int)nP;
    if (n_depth) *n_depth = (int)nD;
    if (res_photo) *res_photo = P;
    if (res_depth) *res_depth = D;
    return std::sqrt(P / nD) + std::sqrt(D / nD);                    // :760-762
}

// calcHessGrad (:767-1100)
void hessgrad_pin(const orc_level* L, const Lut& lut, const Intr& I, const float pose[16], int method,
                  const orc_icp_params* p, double H[36], double g[6], int* n_visible) {
    const int nRows = L->rows, nCols = L->cols;
    const float stdDevPhoto_inv = 1. / p->std_dev_photo;
    const long N = (long)nRows * nCols;
    const bool photo = (method == ORC_PHOTO || method == ORC_PHOTO_DEPTH);
    const bool depth = (method == ORC_DEPTH || method == ORC_PHOTO_DEPTH);
    double acc[27] = {0};
    long nvis = 0;
    #pragma omp parallel
    {
        double a[27] = {0};
        long lv = 0;
        auto add = [&](const float J[6], float r) {
            int k = 0;
            for (int u = 0; u < 6; ++u)
                for (int v = u; v < 6; ++v) a[k++] += (double)(J[u] * J[v]);
            for (int u = 0; u < 6; ++u) a[21 + u] += (double)(J[u] * r);
        };
        #pragma omp for schedule(static)
        for (long i = 0; i < N; ++i) {
            if (lut.x[i] == INVALID_POINT) continue;
            const PP o = project(pose, lut, i, I, nRows, nCols);
            if (!o.vis) continue;
            ++lv;
            const float X = o.X, Y = o.Y, inv = o.inv;
            // jacobianWarpRt (:993-1010)
            float Jw[2][6];
            Jw[0][0] = I.fx * inv;                 Jw[1][0] = 0;
            Jw[0][1] = 0;                          Jw[1][1] = I.fy * inv;
            const float inv2 = inv * inv;
            Jw[0][2] = -I.fx * X * inv2;           Jw[1][2] = -I.fy * Y * inv2;
            Jw[0][3] = -I.fx * Y * X * inv2;       Jw[1][3] = -I.fy * (1 + Y * Y * inv2);
            Jw[0][4] = I.fx * (1 + X * X * inv2);  Jw[1][4] = I.fy * X * Y * inv2;
            Jw[0][5] = -I.fx * Y * inv;            Jw[1][5] = I.fy * X * inv;
            const size_t t = (size_t)o.r * nCols + o.c;
            float Jp[6], rp = 0.f, Jd[6], rd = 0.f;
            bool has_d = false;
            if (photo) {
                const float gx = L->gx[t], gy = L->gy[t];
                if (std::fabs(gx) < p->thres_sal_int && std::fabs(gy) < p->thres_sal_int) continue;   // :1031-1032
                const float photoDiff = L->gray_trg[t] - L->gray_src[i];
                const float w = orc_huber(photoDiff, p->std_dev_photo) * stdDevPhoto_inv;
                rp = w * photoDiff;
                const float wgx = w * gx, wgy = w * gy;                   // (w * grad) * Jw (:1045)
                for (int c = 0; c < 6; ++c) Jp[c] = wgx * Jw[0][c] + wgy * Jw[1][c];
            }
            if (depth) {
                const float dgx = L->dgx[t], dgy = L->dgy[t];
                if (std::fabs(dgx) < p->thres_sal_depth && std::fabs(dgy) < p->thres_sal_depth) continue;  // :1056-1057
                const float depth2 = L->depth_trg[t];
                if (std::isfinite(depth2)) {
                    const float depthDiff = depth2 - o.Z;
                    const float sd = p->std_dev_depth * o.Z;
                    const float w = orc_huber(depthDiff, sd) / sd;
                    rd = w * depthDiff;
                    const float jz[6] = {0, 0, 1, Y, -X, 0};                  // jacobianRt_z (:1072)
                    for (int c = 0; c < 6; ++c) Jd[c] = w * ((dgx * Jw[0][c] + dgy * Jw[1][c]) - jz[c]);
                    has_d = true;
                }
            }
            if (photo) add(Jp, rp);
            if (has_d) add(Jd, rd);
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
    if (n_visible) *n_visible = (int)nvis;
}

}  // namespace

extern "C" double orc_error_pinhole(const orc_level* L, const orc_pinhole* K, int level, const float pose[16],
                                    int method, const orc_icp_params* p, int* n_photo, int* n_depth,
                                    double* res_photo, double* res_depth) {
    const Intr I = level_intrinsics(K, level);
    Lut lut;
    build_lut(L, I, p->min_depth, p->max_depth, lut);
    return error_pin(L, lut, I, pose, method, p, n_photo, n_depth, res_photo, res_depth);
}

extern "C" void orc_hessgrad_pinhole(const orc_level* L, const orc_pinhole* K, int level, const float pose[16],
                                     int method, const orc_icp_params* p, double H[36], double g[6],
                                     int* n_visible) {
    const Intr I = level_intrinsics(K, level);
    Lut lut;
    build_lut(L, I, p->min_depth, p->max_depth, lut);
    hessgrad_pin(L, lut, I, pose, method, p, H, g, n_visible);
}

// alignFrames (:4254-4512), occlusion 0, preceded by setTargetFrame / setSourceFrame (:480-516) on one
// sensor's raw images.  Levenberg-Marquardt constants are the function's own: lambda 0.01, step 10,
// one LM retry, maxIters 10, tol_residual = tol_update = 1e-4 (:4301-4312); CPose3D::exp is the true
// SE(3) exponential here (:4358, no pseudo flag).
extern "C" int orc_align_pinhole(const uint8_t* trg_bgr, const uint16_t* trg_depth, const uint8_t* src_bgr,
                                 const uint16_t* src_depth, int rows, int cols, const orc_pinhole* K,
                                 const float init[16], int method, const orc_icp_params* p, float pose_out[16],
                                 float H_out[36], float g_out[6], orc_icp_stats* st) {
    const int nL = p->n_pyr;
    std::vector<int> R(nL), C(nL);
    std::vector<std::vector<float>> gs(nL), ds(nL), gt(nL), dt(nL), gx(nL), gy(nL), dgx(nL), dgy(nL);
    for (int l = 0; l < nL; ++l) {
        R[l] = l ? R[l - 1] / 2 : rows; C[l] = l ? C[l - 1] / 2 : cols;
        const size_t n = (size_t)R[l] * C[l];
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
    float pose[16];
    memcpy(pose, init, sizeof(pose));
    float Hf[36] = {0}, gf[6] = {0};
    const double step = 10, tol_residual = 1e-4, tol_update = 1e-4;
    const int maxIters = 10;
    auto norm6 = [](const float* u) { float s = 0; for (int k = 0; k < 6; ++k) s += u[k] * u[k]; return std::sqrt(s); };
    // x = -(H + lam*diag H)^-1 g on the float matrices (lam enters as float: Eigen's scalar product)
    auto solve = [&](float lam, float upd[6]) {
        double Hd[36], gd[6], x[6];
        for (int k = 0; k < 36; ++k) Hd[k] = Hf[k];
        for (int k = 0; k < 6; ++k) { Hd[k * 7] = (float)(Hf[k * 7] + lam * Hf[k * 7]); gd[k] = gf[k]; }
        solve6(Hd, gd, x);
        for (int k = 0; k < 6; ++k) upd[k] = (float)x[k];
    };
    auto candidate = [&](const float upd[6], float cand[16]) {
        double ud[6];
        for (int k = 0; k < 6; ++k) ud[k] = upd[k];
        float E[16];
        orc_exp_se3(ud, 0, E);
        matmul4f(E, pose, cand);
    };
    int ret = 0;
    double av[2] = {0, 0}, av_t[2] = {0, 0};
    float av_res = 0.f, av_res_t = 0.f;
    bool have_t = false;
    const bool trace = getenv("R360_ORACLE_TRACE") != nullptr;   // debugging aid: LM trace on stderr
    for (int l = nL - 1; l >= 0; --l) {
        orc_level L = {R[l], C[l], gs[l].data(), ds[l].data(), gt[l].data(), dt[l].data(),
                       gx[l].data(), gy[l].data(), dgx[l].data(), dgy[l].data()};
        const Intr I = level_intrinsics(K, l);
        Lut lut;
        build_lut(&L, I, p->min_depth, p->max_depth, lut);
        double lambda = 0.01;
        int it = 0, evals = 0;
        float upd[6] = {1, 1, 1, 1, 1, 1};
        // the members errorPhotoICP assigns (:759-762) and alignFrames' copies of them (:4329-4332)
        auto eval = [&](const float* P) {
            int nP = 0, nD = 0;
            double rp = 0, rd = 0;
            const double e = error_pin(&L, lut, I, P, method, p, &nP, &nD, &rp, &rd);
            av[0] = std::sqrt(rp / nD);
            av[1] = std::sqrt(rd / nD);
            av_res = (float)(av[0] + av[1]);
            return e;
        };
        double error = eval(pose);
        double diff_error = error;
        while (it < maxIters && norm6(upd) > tol_update && diff_error > tol_residual) {   // :4324
            av_t[0] = av[0]; av_t[1] = av[1]; av_res_t = av_res; have_t = true;
            double H[36], g[6];
            hessgrad_pin(&L, lut, I, pose, method, p, H, g, nullptr);
            for (int k = 0; k < 36; ++k) Hf[k] = (float)H[k];
            for (int k = 0; k < 6; ++k) gf[k] = (float)g[k];
            double HL[36];
            for (int k = 0; k < 36; ++k) HL[k] = Hf[k];
            for (int k = 0; k < 6; ++k) HL[k * 7] = (float)(Hf[k * 7] + (float)lambda * Hf[k * 7]);
            if (rank6(HL) != 6) {                                                          // :4345-4353
                memcpy(pose_out, pose, sizeof(pose));
                if (st) {
                    st->illposed = 1; st->iters[l] = it; st->evals[l] = evals;
                    st->av_photo_residual = av[0]; st->av_depth_residual = av[1]; st->av_residual = av_res;
                    st->residuals_set = 3;
                }
                ret = 1;
                goto done;
            }
            solve(0.f, upd);                                                               // :4355
            float cand[16];
            candidate(upd, cand);                                                          // :4358
            double new_error = eval(cand);
            ++evals;
            diff_error = error - new_error;
            if (trace) fprintf(stderr, "L%d it%d err %.17g new %.17g diff %.3e lam %g |upd| %.3e\n", l, it, error, new_error, diff_error, lambda, (double)norm6(upd));
            if (diff_error > 0) {                                                          // :4374-4380
                lambda /= step;
                memcpy(pose, cand, sizeof(pose));
                error = new_error;
                it = it + 1;
            } else {                                                                       // :4381-4412
                lambda = lambda * step;
                solve((float)lambda, upd);
                candidate(upd, cand);
                new_error = eval(cand);
                ++evals;
                diff_error = error - new_error;
                if (diff_error > 0) {
                    memcpy(pose, cand, sizeof(pose));
                    error = new_error;
                    it = it + 1;
                }
            }
        }
        if (st) { st->iters[l] = it; st->evals[l] = evals; st->error = error; }
    }
    memcpy(pose_out, pose, sizeof(pose));
    if (st && have_t) {                                  // :4507-4509
        st->av_photo_residual = av_t[0]; st->av_depth_residual = av_t[1]; st->av_residual = av_res_t;
        st->residuals_set = 3;
    }
done:
    if (H_out) memcpy(H_out, Hf, sizeof(Hf));
    if (g_out) memcpy(g_out, gf, sizeof(gf));
    return ret;
}
