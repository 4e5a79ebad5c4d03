/* oracle360.h — C ABI of the CPU ORACLE for the rgbd360 registration hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is a plain C++17 restatement of the
 * reference (Dorothy-2016/rgbd360, header-only C++) written for this repository.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it, and only as the checker / the timed CPU baseline.  The product library
 * (rgbd360_amd/lib/librgbd360_hip.so) never links, loads or calls it.
 *
 * Every function cites the reference file:line it restates.  The reference
 * itself cannot be compiled here (Eigen/OpenCV/Boost/PCL/MRPT absent, see
 * DESIGN.md §Oracle), so for the unvendored pieces (OpenCV pyrDown/cvtColor
 * rounding, PCL normals/segmentation/bilateral, MRPT-pbmap) parity is
 * "unpinned": the restatement follows SURVEY.md Appendix C.
 *
 * Conventions: 4x4 poses are float[16] column-major (Eigen default), images are
 * row-major, BGR u8 interleaved, depth u16 millimetres.
 */
#ifndef ORACLE360_H
#define ORACLE360_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_PHOTO = 0, ORC_DEPTH = 1, ORC_PHOTO_DEPTH = 2 };

/* Mirrors RegisterPhotoICP members (include/RegisterPhotoICP.h:119-151,201-221)
 * and the constants of alignFrames360 (:4589-4596). */
typedef struct {
    int    n_pyr;               /* nPyrLevels                          */
    int    max_iters;           /* maxIters per level (10)             */
    float  min_depth;           /* minDepth 0.3                        */
    float  max_depth;           /* maxDepth 6.0                        */
    float  std_dev_photo;       /* stdDevPhoto 6/255 (setGrayVariance) */
    float  std_dev_depth;       /* stdDevDepth 0.2                     */
    float  thres_sal_int;       /* thresSaliencyIntensity 0.01         */
    float  thres_sal_depth;     /* thresSaliencyDepth 0.01             */
    double tol_residual;        /* 1e-3                                */
    double tol_update;          /* 1e-4                                */
    double lambda;              /* 1.0 (only used by the rank test)    */
    int    fixed_iters_level0;  /* 0 = reference schedule; K>0: timing mode, exactly K
                                   candidate evaluations at level 0, no convergence exit */
} orc_icp_params;

typedef struct {
    int    iters[8];            /* num_iterations per level             */
    int    evals[8];            /* error evaluations per level          */
    int    illposed;            /* 1 if the rank test stopped the solve */
    float  sso;                 /* SSO from the last calcHessGrad       */
    double error;               /* last accepted error (level 0)        */
    /* the residual members left after the call (RegisterPhotoICP.h:183-189), as r360_icp_stats */
    double av_photo_residual, av_depth_residual;
    float  av_residual;
    int    residuals_set;       /* bit 0 photo/depth assigned, bit 1 avResidual assigned */
} orc_icp_stats;

/* One pyramid level of the spherical frames (RegisterPhotoICP.h:197-198). */
typedef struct {
    int rows, cols;
    const float *gray_src, *depth_src;
    const float *gray_trg, *depth_trg, *gx, *gy, *dgx, *dgy;
} orc_level;

/* ---- A1: .bin Frame360 archive (Frame360.h:231-266, cvmat_serialization.h:39-55) */
int  orc_bin_dims(const char* path, int* rows, int* cols);
int  orc_bin_load(const char* path, uint8_t* bgr8, uint16_t* depth8);
int  orc_bin_write(const char* path, const uint8_t* bgr8, const uint16_t* depth8, int rows, int cols);

/* ---- A2: CLAMS DiscreteDepthDistortionModel (discrete_depth_distortion_model.cpp) */
void* orc_clams_load(const char* path);          /* load + downsampleParams(2) */
void  orc_clams_free(void* model);
void  orc_clams_undistort(const void* model, float* depth_m, int rows, int cols);
int   orc_clams_export(const void* model, int* hdr /*8*/, float* mult, float* counts);

/* ---- A10: spherical stitching (Frame360.h:386-405, 1099-1148) */
void orc_stitch(const uint8_t* bgr8, const uint16_t* depth8, int rows, int cols,
                const float* rt_inv8 /* 8 x 16 col-major */, const float* K /* 9 col-major */,
                uint8_t* sph_bgr, uint16_t* sph_depth);

/* ---- A14: RegisterPhotoICP pre-processing */
void orc_rgb2gray(const uint8_t* bgr, int n, float* gray);                 /* :485-486 */
void orc_depth_to_m(const uint16_t* d, int n, float* out);                /* :316-317 */
void orc_pyrdown(const float* src, int rows, int cols, float* dst);       /* :292-308 */
void orc_pyr_range(const float* src, int rows, int cols, float min_d, float max_d, float* dst); /* :312-354 */
void orc_gradient(const float* src, int rows, int cols, float* gx, float* gy); /* :365-398 */

/* ---- A16 / A17 */
double orc_error_sphere(const orc_level* L, const float pose[16], int method,
                        const orc_icp_params* p, int* n_valid, double* err2);
void   orc_hessgrad_sphere(const orc_level* L, const float pose[16], int method,
                           const orc_icp_params* p, double H[36], double g[6], int* n_visible);

/* ---- §8(f)1: occlusion-aware variants (occ 1 / 2); occ 0 = the plain functions above */
double orc_error_sphere_occ(const orc_level* L, const float pose[16], int method, int occ,
                            const orc_icp_params* p, int* n_valid);
void   orc_hessgrad_sphere_occ(const orc_level* L, const float pose[16], int method, int occ,
                               const orc_icp_params* p, double H[36], double g[6], int* n_visible);
int    orc_align360_occ(const uint8_t* trg_bgr, const uint16_t* trg_depth,
                        const uint8_t* src_bgr, const uint16_t* src_depth, int rows, int cols,
                        const float init[16], int method, int occlusion, const orc_icp_params* p,
                        float pose_out[16], float H_out[36], float g_out[6], orc_icp_stats* st);

/* ---- A15: full alignFrames360 from sphere images */
int orc_align360(const uint8_t* trg_bgr, const uint16_t* trg_depth,
                 const uint8_t* src_bgr, const uint16_t* src_depth,
                 int rows, int cols, const float init[16], int method,
                 const orc_icp_params* p, float pose_out[16], float H_out[36],
                 float g_out[6], orc_icp_stats* st);

/* ---- §8(f)3: per-sensor pinhole dense path (RegisterPhotoICP.h:560-1100, 4254-4512).
 * Level-0 intrinsics (setCameraMatrix); each level scales them by 1/2^l (:4273-4279). */
typedef struct { float fx, fy, ox, oy; } orc_pinhole;
/* errorPhotoICP -> avResidual (NaN for PHOTO_CONSISTENCY, as the reference: it divides by nValidDepthPts) */
double orc_error_pinhole(const orc_level* L, const orc_pinhole* K, int level, const float pose[16], int method,
                         const orc_icp_params* p, int* n_photo, int* n_depth, double* res_photo, double* res_depth);
void   orc_hessgrad_pinhole(const orc_level* L, const orc_pinhole* K, int level, const float pose[16], int method,
                            const orc_icp_params* p, double H[36], double g[6], int* n_visible);
/* alignFrames (occlusion 0) on one sensor's raw images; params: n_pyr, depth range, std devs and
 * saliency thresholds (the LM constants are alignFrames' own).  Returns 1 when ILL-POSED. */
int    orc_align_pinhole(const uint8_t* trg_bgr, const uint16_t* trg_depth, const uint8_t* src_bgr,
                         const uint16_t* src_depth, int rows, int cols, const orc_pinhole* K,
                         const float init[16], int method, const orc_icp_params* p, float pose_out[16],
                         float H_out[36], float g_out[6], orc_icp_stats* st);

/* ---- A18: CPose3D::exp(mu, pseudo) */
void orc_exp_se3(const double mu[6], int pseudo, float T[16]);

/* glibc std::asin(float) / std::atan2(float,float) — what the reference's projection calls */
void orc_libm(const float* x, const float* y, const float* z, int n, float* asin_out, float* atan2_out);

/* Huber weight (RegisterPhotoICP.h:545-554), float instantiation */
/* ---- A19: RegisterDensePhotoICP (RegisterRGBD360.h:344-520) with calcPhotoICPError_robot
 * (RegisterPhotoICP.h:4905-5076) / calcHessianGradient_robot (:5083-5407).  rows0/cols0 = level-0 image
 * size (camIntrinsicMat).  Returns error2; photo/depth parts and {visible, depth terms} on the side. */
double orc_error_robot(const orc_level* L, int rows0, int cols0, int level, const float pose[16],
                       const float rt[16], const float rt_inv[16], int method, const orc_icp_params* p,
                       double* photo_sum, double* depth_sum, int counts[2]);
/* Hf / gf: float accumulation in raster order (the reference's); Hd / gd: the same terms summed in double. */
void   orc_hessgrad_robot(const orc_level* L, int rows0, int cols0, int level, const float pose[16],
                          const float rt[16], const float rt_inv[16], int method, const orc_icp_params* p,
                          float Hf[36], float gf[6], double Hd[36], double gd[6], int* n_vis);
typedef struct {
    double error[8];
    int    ran[8], iters[8];
    int    illposed_level, info_set;
    float  gradient[6];
} orc_dense_stats;
/* frame1 = target, frame2 = source; [8][rows][cols](x3) raw images; returns 1 (true) / 0 (ILL-POSED). */
int    orc_register_dense_robot(const uint8_t* bgr1, const uint16_t* dep1, const uint8_t* bgr2,
                                const uint16_t* dep2, int rows, int cols, const float* rt8, const float* rt_inv8,
                                const float init[16], int method, const orc_icp_params* p, float pose_out[16],
                                float info_out[36], orc_dense_stats* st);

float orc_huber(float err, float reg);

/* =============================== plane half (A3-A9, A11-A13) ===============================
 * Organized clouds are w x h = (cols/2) x (rows/2) per sensor, row-major:
 *   xyz4[i] = {x, y, z, 0} float, rgb4[i] = {r, g, b, 0} u8, nrm4[i] = {nx, ny, nz, 0}. */

/* A3: CloudRGBD_Ext::getPointCloudUndist (CloudRGBD_Ext.h:78-139) + DownsampleRGBD(2)::
 * downsamplePointCloud (DownsampleRGBD.h:209-311) of one sensor. */
void orc_cloud_downsample(const float* depth_m, const uint8_t* bgr, int rows, int cols,
                          float* xyz4, uint8_t* rgb4);
/* A4: pcl::FastBilateralFilter, sigma_s 10, sigma_r 0.05 (Frame360.h:493-499) */
void orc_bilateral(float* xyz4, int w, int h);
/* A6: pcl::IntegralImageNormalEstimation AVERAGE_3D_GRADIENT, maxDepthChangeFactor 0.02,
 * smoothing 8, depth dependent (Frame360.h:945-955).  dist = distance map. */
void orc_normals(const float* xyz4, int w, int h, float* nrm4, float* dist);

/* A7: one PlanarRegion of OrganizedMultiPlaneSegmentation::segmentAndRefine (App. C.2). */
typedef struct {
    int   label;          /* CCL label (= index into label_indices)                  */
    int   count;          /* inliers after refinement                                */
    int   start_idx;      /* inlier_indices[i].indices[0]                            */
    int   n_contour;      /* boundary length; indices at contour[contour_off ...]    */
    int   contour_off;
    float centroid[3];    /* pre-refinement statistics (PlanarRegion)                */
    float cov[9];
    float model[4];       /* ModelCoefficients (n, d)                                */
    float curvature;
} orc_region;

/* Returns the number of regions, or -1 if max_regions / contour_cap is too small.
 * labels_ccl: CCL labels (-1 = none); labels_final: labels after refinement. */
int orc_segment(const float* xyz4, const float* nrm4, int w, int h,
                int* labels_ccl, int* labels_final,
                orc_region* regions, int max_regions, int* contour, int contour_cap);

/* A8/A9: one PbMap plane (mrpt::pbmap::Plane fields used on the path). */
typedef struct {
    float normal[3], center[3], d, area, elongation, curvature, ppal[3], nrgb[3], intensity;
    int   id, sensor, n_inliers, n_hull;
} orc_plane;

/* PbMap of a frame from per-sensor segmentations (regions packed sensor after sensor,
 * contour_base[s] = offset of sensor s in contour_all). rt8 = Rt_k col-major. */
void* orc_pbmap_from_segments(int n_sensors, int w, int h, const float* xyz4_all, const uint8_t* rgb4_all,
                              const int* labels_final_all, const orc_region* regions, const int* n_regions,
                              const int* contour_all, const int* contour_base, const float* rt8);
/* Whole plane half of one frame: depth_m8 = 8 undistorted depth images (metres), bgr8 = 8 BGR. */
void* orc_pbmap_build(const float* depth_m8, const uint8_t* bgr8, int rows, int cols, const float* rt8);
void  orc_pbmap_free(void* h);
int   orc_pbmap_count(const void* h);
int   orc_pbmap_get(const void* h, int i, orc_plane* out, float* hull_xyz, int hull_cap);
/* SubgraphMatcher thresholds: the [global]/[unary]/[binary] keys of config_files/configLocaliser_*.ini
 * (RegisterRGBD360.h:97-100); angles in degrees.  NULL = configLocaliser_sphericalOdometry.ini. */
typedef struct {
    int   min_planes_recognition;
    float dist_d, angle, color_threshold, intensity_threshold, elongation_threshold, area_threshold;
    float dist_threshold, angle_threshold, height_threshold, cos_angle_parallel, planar_normal_angle;
    long  max_nodes;
} orc_match_params;
/* A11+A12 tables: subgraph ids, unary [ns][nt] and binary [(i*nt+j)][words] bitsets; returns words. */
int   orc_match_tables(const void* href, const void* htrg, size_t max_match_planes, int mode, int* ns, int* nt,
                       int* sid, int* tid, uint8_t* unary, uint64_t* binary, int cap, const orc_match_params* mp);
/* A11-A13: RegisterRGBD360::RegisterPbMap.  Returns 1 good, 0 insufficient / ill-conditioned. */
int   orc_register_pbmap(const void* href, const void* htrg, size_t max_match_planes, int mode, float pose[16],
                         float info[36], int* pairs, int pair_cap, int* n_match, float* area_matched,
                         float* area_src, float* area_trg, const orc_match_params* mp);
/* Nodes the calling thread's last orc_register_pbmap search visited and whether the node budget stopped it. */
void  orc_last_match_stats(long* nodes, int* truncated);
/* The interpretation tree alone over given tables; returns 1 if max_nodes stopped it. */
int   orc_tree_search(int ns, int nt, const uint8_t* unary, const uint64_t* binary, int words, const double* area,
                      long max_nodes, int* best, long* nodes);

#ifdef __cplusplus
}
#endif
#endif
