// robot_oracle.cpp — ORACLE (test infrastructure only, see oracle360.h).
// RegisterRGBD360::RegisterDensePhotoICP, the per-sensor pinhole dense registration
// of two Frame360s in the rig ("robot") frame —
//   RegisterDensePhotoICP       include/RegisterRGBD360.h:344-520
//   calcPhotoICPError_robot     include/RegisterPhotoICP.h:4905-5076 (all-pixel branch)
//   calcHessianGradient_robot   :5083-5407                            (all-pixel branch)
// restated literally: serial raster loops (the inner OpenMP loop runs nested inside the per-sensor
// parallel region, i.e. on one thread; calcHessianGradient_robot's is commented out), float hessian /
// gradient accumulation in raster order, the LM loop as written — including the "new" error evaluated
// at pose_estim (:430-432, :467-469), which makes the candidate never accepted.  Sensor errors are summed
// in sensor order (the reference's OpenMP reduction order is unspecified).  jacobianRt_z (:5372) is
// uninitialised in the reference and taken as zero (documented in DESIGN.md).
#include "oracle360.h"
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle_la.h"

namespace {

struct V4 { float x, y, z, w; };

// Eigen Matrix4f * Vector4f, col-major
inline V4 xform(const float* M, float x, float y, float z, float w) {
    V4 o;
    o.x = M[0] * x + M[4] * y + M[8] * z + M[12] * w;
    o.y = M[1] * x + M[5] * y + M[9] * z + M[13] * w;
    o.z = M[2] * x + M[6] * y + M[10] * z + M[14] * w;
    o.w = M[3] * x + M[7] * y + M[11] * z + M[15] * w;
    return o;
}

// camIntrinsicMat of RegisterDensePhotoICP (RegisterRGBD360.h:357-365), from the level-0 image size
struct Cam { float f, ox, oy; };
Cam cam_of(int rows0, int cols0) {
    const float img_width = (float)cols0, img_height = (float)rows0;
    const float res_factor_VGA = img_width / 640.0;
    Cam c;
    c.f = 525 * res_factor_VGA;
    c.ox = img_width / 2 - 0.5;
    c.oy = img_height / 2 - 0.5;
    return c;
}

double error_robot(const orc_level* L, const Cam& K, int level, const float pose[16], const float rt[16],
                   const float rt_inv[16], int method, const orc_icp_params* p, double* photo_sum, double* depth_sum,
                   int counts[2]) {
    double error2 = 0.0, eP = 0.0, eD = 0.0;
    const int nRows = L->rows, nCols = L->cols;
    const float scaleFactor = 1.0 / pow(2, level);                               // :4917-4924
    const float fx = K.f * scaleFactor, fy = K.f * scaleFactor;
    const float ox = K.ox * scaleFactor, oy = K.oy * scaleFactor;
    const float inv_fx = 1. / fx, inv_fy = 1. / fy;
    float tmp[16], relPoseCam[16];
    matmul4f(rt_inv, pose, tmp);                                                 // :4926-4927
    matmul4f(tmp, rt, relPoseCam);
    const float stdDevPhoto = p->std_dev_photo, stdDevDepth = p->std_dev_depth;
    const double stdDevPhoto_inv = 1. / stdDevPhoto;
    int nvis = 0, ndep = 0;
    for (int r = 0; r < nRows; r++)
        for (int c = 0; c < nCols; c++) {
            const size_t i = (size_t)r * nCols + c;
            float pz = L->depth_src[i];
            if (!(p->min_depth < pz && pz < p->max_depth)) continue;
            const float px = (c - ox) * pz * inv_fx;
            const float py = (r - oy) * pz * inv_fy;
            const V4 t = xform(relPoseCam, px, py, pz, 1.f);
            const double inv_transformedPz = 1.0 / t.z;
            const double transformed_c = (t.x * fx) * inv_transformedPz + ox;
            const double transformed_r = (t.y * fy) * inv_transformedPz + oy;
            const double rr = round(transformed_r), cc = round(transformed_c);
            // (int)round() then the bounds test; NaN / huge values convert to INT_MIN on x86
            if (!(rr >= 0 && rr < nRows && cc >= 0 && cc < nCols)) continue;
            const size_t ti = (size_t)(int)rr * nCols + (int)cc;
            ++nvis;
            if (method == ORC_PHOTO || method == ORC_PHOTO_DEPTH) {
                const float pixel1 = L->gray_src[i], pixel2 = L->gray_trg[ti];
                const float photoDiff = pixel2 - pixel1;
                const double weight_photo = orc_huber(photoDiff, stdDevPhoto) * stdDevPhoto_inv;
                const float weightedErrorPhoto = weight_photo * photoDiff;
                error2 += weightedErrorPhoto * weightedErrorPhoto;
                eP += weightedErrorPhoto * weightedErrorPhoto;
            }
            if (method == ORC_DEPTH || method == ORC_PHOTO_DEPTH) {
                const float depth2 = L->depth_trg[ti];
                if (std::isfinite(depth2)) {
                    const float depth1 = L->depth_src[i];
                    const float depthDiff = depth2 - depth1;
                    const float stdDev_depth1 = stdDevDepth * depth1;
                    const double weight_depth = orc_huber(depthDiff, stdDev_depth1) / stdDev_depth1;
                    const float weightedErrorDepth = weight_depth * depthDiff;
                    error2 += weightedErrorDepth * weightedErrorDepth;
                    eD += weightedErrorDepth * weightedErrorDepth;
                    ++ndep;
                }
            }
        }
    if (photo_sum) *photo_sum = eP;
    if (depth_sum) *depth_sum = eD;
    if (counts) { counts[0] = nvis; counts[1] = ndep; }
    return error2;
}

// hessian / gradient as the reference accumulates them (float, raster order) in Hf / gf, and the
// same float terms summed in double in Hd / gd
void hessgrad_robot(const orc_level* L, const Cam& K, int level, const float pose[16], const float rt[16],
                    const float rt_inv[16], int method, const orc_icp_params* p, float Hf[36], float gf[6],
                    double Hd[36], double gd[6], int* n_vis) {
    const int nRows = L->rows, nCols = L->cols;
    const double scaleFactor = 1.0 / pow(2, level);                              // :5093-5099
    const double fx = K.f * scaleFactor, fy = K.f * scaleFactor;
    const double ox = K.ox * scaleFactor, oy = K.oy * scaleFactor;
    const double inv_fx = 1. / fx, inv_fy = 1. / fy;
    const float stdDevPhoto = p->std_dev_photo, stdDevDepth = p->std_dev_depth;
    const double stdDevPhoto_inv = 1. / stdDevPhoto;
    const bool photo = (method == ORC_PHOTO || method == ORC_PHOTO_DEPTH);
    const bool depth = (method == ORC_DEPTH || method == ORC_PHOTO_DEPTH);
    for (int k = 0; k < 36; ++k) { Hf[k] = 0.f; Hd[k] = 0.0; }
    for (int k = 0; k < 6; ++k) { gf[k] = 0.f; gd[k] = 0.0; }
    int nvis = 0;
    auto add = [&](const float J[6], float res) {
        for (int a = 0; a < 6; ++a) {
            for (int b = 0; b < 6; ++b) {
                const float t = J[a] * J[b];
                Hf[a * 6 + b] += t;
                Hd[a * 6 + b] += t;
            }
            const float t = J[a] * res;
            gf[a] += t;
            gd[a] += t;
        }
    };
    for (int r = 0; r < nRows; r++)
        for (int c = 0; c < nCols; c++) {
            const size_t i = (size_t)r * nCols + c;
            const float pz = L->depth_src[i];
            if (!(p->min_depth < pz && pz < p->max_depth)) continue;
            const float px = (c - ox) * pz * inv_fx;
            const float py = (r - oy) * pz * inv_fy;
            const V4 p1 = xform(rt, px, py, pz, 1.f);                            // point3D_robot
            const V4 p2 = xform(pose, p1.x, p1.y, p1.z, p1.w);                  // point3D_robot2
            const V4 t = xform(rt_inv, p2.x, p2.y, p2.z, p2.w);                 // transformedPoint3D
            const double inv_transformedPz = 1.0 / t.z;
            const double transformed_c = (t.x * fx) * inv_transformedPz + ox;
            const double transformed_r = (t.y * fy) * inv_transformedPz + oy;
            const double rr = round(transformed_r), cc = round(transformed_c);
            if (!(rr >= 0 && rr < nRows && cc >= 0 && cc < nCols)) continue;
            const size_t ti = (size_t)(int)rr * nCols + (int)cc;
            ++nvis;
            // jacobianT36 = Rinv * [I | -skew(point3D_robot2)] (:5289-5292)
            float S[3][6];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) S[a][b] = (a == b) ? 1.f : 0.f;
            S[0][3] = 0;      S[0][4] = p2.z;   S[0][5] = -p2.y;
            S[1][3] = -p2.z;  S[1][4] = 0;      S[1][5] = p2.x;
            S[2][3] = p2.y;   S[2][4] = -p2.x;  S[2][5] = 0;
            float T36[3][6];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 6; ++b)
                    T36[a][b] = rt_inv[a] * S[0][b] + rt_inv[4 + a] * S[1][b] + rt_inv[8 + a] * S[2][b];
            float P23[2][3];                                                     // :5294-5303
            P23[0][0] = fx * inv_transformedPz; P23[1][0] = 0;
            P23[0][1] = 0;                      P23[1][1] = fy * inv_transformedPz;
            P23[0][2] = -fx * t.x * inv_transformedPz * inv_transformedPz;
            P23[1][2] = -fy * t.y * inv_transformedPz * inv_transformedPz;
            float Jw[2][6];
            for (int a = 0; a < 2; ++a)
                for (int b = 0; b < 6; ++b)
                    Jw[a][b] = P23[a][0] * T36[0][b] + P23[a][1] * T36[1][b] + P23[a][2] * T36[2][b];
            float Jp[6], Jd[6];
            double weightedErrorPhoto = 0, weightedErrorDepth = 0;
            float depth2 = 0;
            if (photo) {
                const float pixel1 = L->gray_src[i];
                const float gx = L->gx[ti], gy = L->gy[ti];
                if (std::fabs(gx) < p->thres_sal_int && std::fabs(gy) < p->thres_sal_int) continue;  // :5319
                const float pixel2 = L->gray_trg[ti];
                const float photoDiff = pixel2 - pixel1;
                const double weight_photo = orc_huber(photoDiff, stdDevPhoto) * stdDevPhoto_inv;
                weightedErrorPhoto = weight_photo * photoDiff;
                const float wf = (float)weight_photo;                            // Eigen: float scalar
                const float wg0 = wf * gx, wg1 = wf * gy;
                for (int b = 0; b < 6; ++b) Jp[b] = wg0 * Jw[0][b] + wg1 * Jw[1][b];
            }
            if (depth) {
                depth2 = L->depth_trg[ti];
                const float depth1 = L->depth_src[i];
                const float dgx = L->dgx[ti], dgy = L->dgy[ti];
                if (std::fabs(dgx) < p->thres_sal_depth && std::fabs(dgy) < p->thres_sal_depth) continue;  // :5348
                const float depthDiff = depth2 - depth1;
                const float stdDev_depth1 = stdDevDepth * depth1;
                const double weight_depth = orc_huber(depthDiff, stdDev_depth1) / stdDev_depth1;
                weightedErrorDepth = weight_depth * depthDiff;
                const float jacobianRt_z[6] = {0, 0, 0, 0, 0, 0};                 // uninitialised in the reference
                for (int b = 0; b < 6; ++b)
                    Jd[b] = (float)weight_depth * ((dgx * Jw[0][b] + dgy * Jw[1][b]) - jacobianRt_z[b]);
            }
            if (photo) add(Jp, (float)weightedErrorPhoto);                     // :5375-5383
            if (depth && std::isfinite(depth2)) add(Jd, (float)weightedErrorDepth);
        }
    if (n_vis) *n_vis = nvis;
}

struct SensorPyr {
    std::vector<int> R, C;
    std::vector<std::vector<float>> gs, ds, gt, dt, gx, gy, dgx, dgy;
    orc_level level(int l) const {
        return orc_level{R[l], C[l], gs[l].data(), ds[l].data(), gt[l].data(), dt[l].data(),
                         gx[l].data(), gy[l].data(), dgx[l].data(), dgy[l].data()};
    }
};

// setTargetFrame / setSourceFrame (RegisterPhotoICP.h:480-516) on one sensor's raw images
void build_pyr(const uint8_t* trg_bgr, const uint16_t* trg_depth, const uint8_t* src_bgr, const uint16_t* src_depth,
               int rows, int cols, int nL, const orc_icp_params* p, SensorPyr& P) {
    P.R.resize(nL); P.C.resize(nL);
    for (auto* v : {&P.gs, &P.ds, &P.gt, &P.dt, &P.gx, &P.gy, &P.dgx, &P.dgy}) v->resize(nL);
    for (int l = 0; l < nL; ++l) {
        P.R[l] = l ? P.R[l - 1] / 2 : rows; P.C[l] = l ? P.C[l - 1] / 2 : cols;
        const size_t n = (size_t)P.R[l] * P.C[l];
        for (auto* v : {&P.gs, &P.ds, &P.gt, &P.dt, &P.gx, &P.gy, &P.dgx, &P.dgy}) (*v)[l].resize(n);
    }
    orc_rgb2gray(src_bgr, rows * cols, P.gs[0].data());
    orc_rgb2gray(trg_bgr, rows * cols, P.gt[0].data());
    orc_depth_to_m(src_depth, rows * cols, P.ds[0].data());
    orc_depth_to_m(trg_depth, rows * cols, P.dt[0].data());
    for (int l = 1; l < nL; ++l) {
        orc_pyrdown(P.gs[l - 1].data(), P.R[l - 1], P.C[l - 1], P.gs[l].data());
        orc_pyrdown(P.gt[l - 1].data(), P.R[l - 1], P.C[l - 1], P.gt[l].data());
        orc_pyr_range(P.ds[l - 1].data(), P.R[l - 1], P.C[l - 1], p->min_depth, p->max_depth, P.ds[l].data());
        orc_pyr_range(P.dt[l - 1].data(), P.R[l - 1], P.C[l - 1], p->min_depth, p->max_depth, P.dt[l].data());
    }
    for (int l = 0; l < nL; ++l) {
        orc_gradient(P.gt[l].data(), P.R[l], P.C[l], P.gx[l].data(), P.gy[l].data());
        orc_gradient(P.dt[l].data(), P.R[l], P.C[l], P.dgx[l].data(), P.dgy[l].data());
    }
}

}  // namespace

extern "C" double orc_error_robot(const orc_level* L, int rows0, int cols0, int level, const float pose[16],
                                  const float rt[16], const float rt_inv[16], int method, const orc_icp_params* p,
                                  double* photo_sum, double* depth_sum, int counts[2]) {
    return error_robot(L, cam_of(rows0, cols0), level, pose, rt, rt_inv, method, p, photo_sum, depth_sum, counts);
}

extern "C" void orc_hessgrad_robot(const orc_level* L, int rows0, int cols0, int level, const float pose[16],
                                   const float rt[16], const float rt_inv[16], int method, const orc_icp_params* p,
                                   float Hf[36], float gf[6], double Hd[36], double gd[6], int* n_vis) {
    hessgrad_robot(L, cam_of(rows0, cols0), level, pose, rt, rt_inv, method, p, Hf, gf, Hd, gd, n_vis);
}

// RegisterDensePhotoICP(frame1, frame2, pose_estim, method) (RegisterRGBD360.h:344-520); frame1 = the
// target of every sensor's alignment, frame2 the source.  bgr / depth: [8][rows][cols](x3).
extern "C" int orc_register_dense_robot(const uint8_t* bgr1, const uint16_t* dep1, const uint8_t* bgr2,
                                        const uint16_t* dep2, int rows, int cols, const float* rt8,
                                        const float* rt_inv8, const float init[16], int method,
                                        const orc_icp_params* p, float pose_out[16], float info_out[36],
                                        orc_dense_stats* st) {
    const int nL = p->n_pyr;
    const Cam K = cam_of(rows, cols);
    std::vector<SensorPyr> S(8);
    const size_t n0 = (size_t)rows * cols;
    #pragma omp parallel for num_threads(8)
    for (int k = 0; k < 8; ++k)
        build_pyr(bgr1 + k * n0 * 3, dep1 + k * n0, bgr2 + k * n0 * 3, dep2 + k * n0, rows, cols, nL, p, S[k]);
    if (st) { memset(st, 0, sizeof(*st)); st->illposed_level = -1; }
    float pose_estim[16];
    memcpy(pose_estim, init, sizeof(pose_estim));
    float Hessian[36] = {0}, Gradient[6] = {0};    // uninitialised in the reference until a loop runs
    bool hess_set = false;
    auto total_error = [&](int l, const float* pose) {
        double e[8];
        #pragma omp parallel for num_threads(8)
        for (int k = 0; k < 8; ++k) {
            const orc_level L = S[k].level(l);
            e[k] = error_robot(&L, K, l, pose, rt8 + 16 * k, rt_inv8 + 16 * k, method, p, nullptr, nullptr, nullptr);
        }
        double error = 0.0;
        for (int k = 0; k < 8; ++k) error += e[k];
        return error;
    };
    auto solve_update = [&](double lambda, float upd[6]) {   // -(H + lambda diag H)^-1 g
        double Hl[36], gd[6], x[6];
        for (int k = 0; k < 36; ++k) Hl[k] = Hessian[k];
        for (int k = 0; k < 6; ++k) { Hl[k * 7] = (float)(Hessian[k * 7] + (float)lambda * Hessian[k * 7]); gd[k] = Gradient[k]; }
        solve6(Hl, gd, x);
        for (int k = 0; k < 6; ++k) upd[k] = (float)x[k];
    };
    auto candidate = [&](const float upd[6], float cand[16]) {
        double ud[6];
        for (int k = 0; k < 6; ++k) ud[k] = upd[k];
        float E[16];
        orc_exp_se3(ud, 0, E);                     // CPose3D::exp, pseudo_exponential = false
        matmul4f(E, pose_estim, cand);
    };
    for (int l = nL - 1; l >= 0; --l) {
        double lambda = 0.001;
        const double step = 10;
        const unsigned LM_maxIters = 1;
        int it = 0;
        const int maxIters = 10;
        const double tol_residual = pow(10, -1), tol_update = pow(10, -6);
        float update_pose[6] = {1, 1, 1, 1, 1, 1};
        auto norm6 = [&]() { float s = 0; for (int k = 0; k < 6; ++k) s += update_pose[k] * update_pose[k]; return std::sqrt(s); };
        double error = total_error(l, pose_estim);
        double diff_error = error;
        if (st) st->error[l] = error;
        while (it < maxIters && norm6() > tol_update && diff_error > tol_residual) {
            if (st) st->ran[l] = 1;
            for (int k = 0; k < 36; ++k) Hessian[k] = 0.f;
            for (int k = 0; k < 6; ++k) Gradient[k] = 0.f;
            float Hk[8][36], gk[8][6];
            #pragma omp parallel for num_threads(8)
            for (int k = 0; k < 8; ++k) {
                const orc_level L = S[k].level(l);
                double Hd[36], gd[6];
                hessgrad_robot(&L, K, l, pose_estim, rt8 + 16 * k, rt_inv8 + 16 * k, method, p, Hk[k], gk[k], Hd, gd,
                               nullptr);
            }
            for (int k = 0; k < 8; ++k) {
                for (int q = 0; q < 36; ++q) Hessian[q] += Hk[k][q];
                for (int q = 0; q < 6; ++q) Gradient[q] += gk[k][q];
            }
            hess_set = true;
            double HL[36];
            for (int k = 0; k < 36; ++k) HL[k] = Hessian[k];
            for (int k = 0; k < 6; ++k) HL[k * 7] = (float)(Hessian[k * 7] + (float)lambda * Hessian[k * 7]);
            if (rank6(HL) != 6) {                                                    // :427-434
                memcpy(pose_out, pose_estim, sizeof(pose_estim));
                if (st) st->illposed_level = l;
                return 0;
            }
            solve_update(lambda, update_pose);                                       // :437
            float pose_estim_temp[16];
            candidate(update_pose, pose_estim_temp);                                 // :439
            double new_error = total_error(l, pose_estim);                           // :430-432 (pose_estim)
            diff_error = error - new_error;
            if (diff_error > 0) {
                lambda /= step;
                memcpy(pose_estim, pose_estim_temp, sizeof(pose_estim));
                error = new_error;
                it = it + 1;
            } else {
                unsigned LM_it = 0;
                while (LM_it < LM_maxIters && diff_error < 0) {
                    lambda = lambda * step;
                    solve_update(lambda, update_pose);
                    candidate(update_pose, pose_estim_temp);
                    new_error = total_error(l, pose_estim);                          // :467-469 (pose_estim)
                    diff_error = error - new_error;
                    if (diff_error > 0) {
                        memcpy(pose_estim, pose_estim_temp, sizeof(pose_estim));
                        error = new_error;
                        it = it + 1;
                    }
                    LM_it = LM_it + 1;
                }
            }
        }
        if (st) st->iters[l] = it;
    }
    memcpy(pose_out, pose_estim, sizeof(pose_estim));
    memcpy(info_out, Hessian, sizeof(Hessian));
    if (st) { st->info_set = hess_set; memcpy(st->gradient, Gradient, sizeof(Gradient)); }
    return 1;
}
