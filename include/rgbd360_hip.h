/* rgbd360_hip.h — C-ABI of librgbd360_hip.so, the MI355X-native (gfx950) implementation of
 * rgbd360's frame-to-frame registration hot path.
 *
 * This is the drop-in boundary.  The reference (Dorothy-2016/rgbd360) has no plugin/FFI layer:
 * its applications instantiate header-only classes directly.  Each entry point
 * below replaces one method of those classes; the C++ façade headers in include/rgbd360/ keep
 * the reference class names and signatures on top of this ABI.
 *
 * Conventions
 *   - 4x4 poses are float[16] COLUMN-major (Eigen default, as Eigen::Matrix4f::data()).
 *     6x6 matrices are float[36] column-major (symmetric ones are identical either way).
 *   - Sensor images: 8 sensors stored contiguously, each rows x cols, BGR u8 interleaved
 *     (as cv::Mat CV_8UC3 in the .bin files) and depth u16 millimetres (CV_16UC1).
 *   - Return codes: 0 = OK, 1 = soft failure (the reference returned false / ill-posed),
 *     < 0 = error (message in r360_last_error(), thread-local).  No exceptions cross the ABI.
 *   - One r360_ctx per (GPU, host thread); a ctx is not thread-safe.  All calls are ordered on
 *     the ctx's HIP stream and synchronous at return unless named *_async.
 */
#ifndef RGBD360_HIP_H
#define RGBD360_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define R360_NUM_SENSORS 8
#define R360_MAX_PYR 6

typedef struct r360_ctx r360_ctx;
typedef struct r360_calib r360_calib;
typedef struct r360_frame r360_frame;

/* ---------------------------------------------------------------- context */
int         r360_ctx_create(int device, r360_ctx** out);
void        r360_ctx_destroy(r360_ctx* ctx);
int         r360_ctx_sync(r360_ctx* ctx);
void*       r360_ctx_stream(r360_ctx* ctx);        /* hipStream_t of the ctx */
const char* r360_last_error(void);
const char* r360_version(void);
/* The shipped data directory (calib/, config_files/, samples/): $R360_DATA_DIR, else <tree>/data of the tree the
 * library sits in — the files the reference finds under PROJECT_SOURCE_PATH (Calib360.h:107, :125). */
const char* r360_data_dir(void);

/* ---------------------------------------------------------------- Calib360
 * Replaces include/Calib360.h:44-132.  rows/cols = per-sensor image size; the pinhole
 * cameraMatrix is f = 525*cols/640, c = (cols/2-0.5, rows/2-0.5), which reproduces the
 * reference's QVGA constant (Calib360.h:73-77) and its commented VGA one (:83-85). */
int  r360_calib_create(r360_ctx* ctx, int rows, int cols, r360_calib** out);
void r360_calib_destroy(r360_calib* c);
/* Rt_[8] (Calib360.h:53), column-major 8 x float[16]; Rt_inv is derived (Calib360.h:129). */
int  r360_calib_set_extrinsics(r360_calib* c, const float* rt8);
int  r360_calib_get_extrinsics(const r360_calib* c, float* rt8, float* rt_inv8, float K[9]);
/* loadExtrinsicCalibration(dir): reads dir/Rt_0{1..8}.txt (Calib360.h:122-131); dir NULL or "" = the shipped
 * r360_data_dir()/calib/Extrinsics (the reference's "" default, :124-125). */
int  r360_calib_load_extrinsics(r360_calib* c, const char* dir);
/* loadIntrinsicCalibration(dir): CLAMS dir/distortion_model{1..8} + downsampleParams(2)
 * (Calib360.h:104-119); dir NULL or "" = r360_data_dir()/calib/Intrinsics (:106-107).  Without intrinsics
 * undistort() is the identity. */
int  r360_calib_load_intrinsics(r360_calib* c, const char* dir);
/* A calibration without sensors for spheres given as images (setSourceFrame / setTargetFrame(cv::Mat&,
 * cv::Mat&), RegisterPhotoICP.h:480-516): the ICP tables of an sph_rows x sph_cols sphere
 * (sph_cols % 8 == 0).  Its frames only take r360_frame_set_sphere. */
int  r360_calib_create_sphere(r360_ctx* ctx, int sph_rows, int sph_cols, r360_calib** out);

/* ---------------------------------------------------------------- Frame360
 * Replaces include/Frame360.h:93-1150. */
enum {
    R360_BUILD_UNDISTORT = 1u << 0,  /* Frame360::undistort()            Frame360.h:293   */
    R360_BUILD_SPHERE    = 1u << 1,  /* Frame360::stitchSphericalImage() Frame360.h:386   */
    R360_BUILD_PYRAMID   = 1u << 2,  /* RegisterPhotoICP::set{Source,Target}Frame :480-516 */
    R360_BUILD_CLOUD     = 1u << 3,  /* Frame360::buildSphereCloud()     Frame360.h:467   */
    R360_BUILD_PLANES    = 1u << 4,  /* Frame360::getPlanes()            Frame360.h:615   */
    R360_BUILD_SENSOR_PYRAMID = 1u << 5, /* per-sensor setSource/TargetFrame (pinhole alignFrames) */
};
int  r360_frame_create(r360_ctx* ctx, const r360_calib* calib, r360_frame** out);
void r360_frame_destroy(r360_frame* f);
/* Host images -> HBM (8 sensors contiguous).  Replaces loadFrame's decode step. */
int  r360_frame_upload(r360_frame* f, const uint8_t* bgr8, const uint16_t* depth8);
/* Same copy, enqueued on the ctx stream without waiting (OdometryRGBD360's per-frame input upload in
 * the pipelined sequence driver).  The host buffers must stay valid until the stream has consumed
 * them; page-locked buffers (r360_host_register) make the copy asynchronous to the host. */
int  r360_frame_upload_async(r360_frame* f, const uint8_t* bgr8, const uint16_t* depth8);
/* setSourceFrame / setTargetFrame(cv::Mat& imgRGB, cv::Mat& imgDepth) (RegisterPhotoICP.h:480-516): the
 * sphere as images (BGR u8 [sph_rows][sph_cols][3], range u16 mm [sph_rows][sph_cols], as sphereRGB /
 * sphereDepth) replaces the frame's and its pyramid is rebuilt.  The size must be the frame's. */
int  r360_frame_set_sphere(r360_frame* f, const uint8_t* bgr, const uint16_t* range_mm, int sph_rows, int sph_cols);
/* Page-lock / release host memory for asynchronous uploads (hipHostRegister). */
int  r360_host_register(void* p, size_t bytes);
int  r360_host_unregister(void* p);
/* Device-resident images (already in HBM on the ctx's device); copied device-to-device. */
int  r360_frame_upload_device(r360_frame* f, const void* d_bgr8, const void* d_depth8);
/* Frame360::loadFrame(path) (Frame360.h:231-266): Boost binary archive of 8 x {RGB, depth} and
 * the timestamp digit matrix (get_uint64_t_ofMatrixRepresentation, SerializeFrameRGBD.h:77-89). */
int  r360_frame_load_bin(r360_frame* f, const char* path);
/* Frame360::serialize(fileName) (Frame360.h:332-345): writes the raw images as loaded/uploaded. */
int  r360_frame_save_bin(r360_frame* f, const char* path);
/* Frame360::setTimeStamp / timeStamp (Frame360.h:181-184). */
int  r360_frame_set_timestamp(r360_frame* f, uint64_t ts);
int  r360_frame_get_timestamp(const r360_frame* f, uint64_t* ts);
int  r360_frame_build(r360_frame* f, unsigned flags);
int  r360_frame_build_async(r360_frame* f, unsigned flags);
/* r360_frame_build of n distinct frames of one device (Frame360::getPlanes of a keyframe batch, Frame360.h:615-640):
 * the plane stages of frames of one size run batched, up to 8 frames per launch of the plane kernels, on the stream
 * of frames[0]'s context; every other stage on each frame's own stream.  Synchronous; each frame's results equal
 * its r360_frame_build's. */
int  r360_frames_build(r360_frame* const* frames, int n, unsigned flags);
int  r360_frame_dims(const r360_frame* f, int* rows, int* cols, int* sph_rows, int* sph_cols);
/* RegisterPhotoICP::setNumPyr (RegisterPhotoICP.h:224-227) for the frame: its pyramid stops at n levels (default:
 * the calibration's full depth).  Alignments of the frame then take nPyr <= n. */
int  r360_frame_set_levels(r360_frame* f, int n);
/* Source-point compaction of the frame's pyramid builds (no reference counterpart: a layout choice).  all = 1
 * (default): every level's valid source pixels are compacted once per build, which a lone alignment's passes read
 * (PF 5).  all = 0: only the levels a batched pass cannot stream as an image are compacted (two launches per build
 * fewer, for frames that only enter batched alignments, e.g. a dense queue's); a lone alignment then streams the
 * images too.  Poses are equal to rounding either way.  Takes effect at the next build. */
int  r360_frame_set_compaction(r360_frame* f, int all);
/* The R360_BUILD_* stages the frame's current images have been through (an upload or load clears them). */
int  r360_frame_built(const r360_frame* f, unsigned* flags);
/* sphereRGB (BGR u8) / sphereDepth (u16 range mm) (Frame360.h:104-107). */
int  r360_frame_get_sphere(r360_frame* f, uint8_t* bgr, uint16_t* depth);
/* Undistorted per-sensor depth in metres (CloudRGBD_Ext::m_depthEigUndistort). */
int  r360_frame_get_depth_m(r360_frame* f, float* depth8);
/* Pyramid level of the frame as RegisterPhotoICP sees it (gray /255, depth m, target
 * gradients with the alignFrames360 seam mask applied).  Any pointer may be NULL. */
int  r360_frame_get_level(r360_frame* f, int level, int* rows, int* cols, float* gray, float* depth,
                          float* gx, float* gy, float* dgx, float* dgy);
/* The level's compacted ICP source points (valid depth, raster order) as {x, y, z, gray} quadruples:
 * LUT_xyz_sphere (RegisterPhotoICP.h:4553-4587) and the gray value.  *n = their count; copies min(n, cap). */
int  r360_frame_get_points(r360_frame* f, int level, float* xyzg, int cap, int* n);
/* Sensor k's pinhole pyramid level (R360_BUILD_SENSOR_PYRAMID; no seam mask). */
int  r360_frame_get_sensor_level(r360_frame* f, int sensor, int level, int* rows, int* cols, float* gray,
                                 float* depth, float* gx, float* gy, float* dgx, float* dgy);

/* ---------------------------------------------------------------- RegisterPhotoICP
 * Replaces include/RegisterPhotoICP.h:85-4784 (spherical path). */
enum { R360_PHOTO_CONSISTENCY = 0, R360_DEPTH_CONSISTENCY = 1, R360_PHOTO_DEPTH = 2 };

typedef struct {
    int    n_pyr;               /* setNumPyr (default 4; odometry apps use 5)  :224      */
    int    max_iters;           /* maxIters per level = 10                     :4593     */
    float  min_depth;           /* setMinDepth 0.3                             :202,230  */
    float  max_depth;           /* setMaxDepth 6.0                             :203,236  */
    float  std_dev_photo;       /* setGrayVariance: stdDevPhoto (6/255)        :208,242  */
    float  std_dev_depth;       /* setDepthVariance: stdDevDepth (0.2)         :211,248  */
    float  thres_sal_int;       /* thresSaliencyIntensity 0.01                 :218      */
    float  thres_sal_depth;     /* thresSaliencyDepth 0.01                     :219      */
    double tol_residual;        /* 1e-3                                        :4594     */
    double tol_update;          /* 1e-4                                        :4595     */
    double lambda;              /* 1.0, rank test only                         :4589     */
    int    fixed_iters_level0;  /* 0: reference schedule.  K>0: benchmark timing mode, exactly
                                   K candidate evaluations at level 0 (no convergence exit). */
} r360_icp_params;

typedef struct {
    int    iters[8];            /* num_iterations per level (:4772)          */
    int    evals[8];            /* candidate evaluations per level           */
    int    illposed;            /* 1: rank(H + lambda diag H) != 6 (:4682)   */
    float  sso;                 /* SSO (:3226)                               */
    double error;               /* accepted error at level 0                 */
    int    passes;              /* fused residual/Jacobian/JtJ passes run     */
    int    persistent;          /* r360_align360: 1 = each level ran as ONE launch (k_icp_level) instead of
                                   one launch per pass; same results either way */
    /* The public residual members RegisterPhotoICP leaves after the call (RegisterPhotoICP.h:183-189).
     * alignFrames360 with occlusion 1 / 2: avPhotoResidual / avDepthResidual of the last error evaluation
     * (errorPhotoICP_sphereOcc1 :3360-3362, Occ2 :3852-3853); avResidual is set only when ILL-POSED (= 0,
     * :4688).  alignFrames360 with occlusion 0 assigns none of them (errorPhotoICP_sphere does not).
     * alignFrames (pinhole): the values copied at the start of the last loop iteration (:4329-4332,
     * :4507-4509; errorPhotoICP :759-762).  residuals_set: bit 0 = avPhotoResidual / avDepthResidual
     * assigned, bit 1 = avResidual assigned; unassigned members keep their previous value in the façades. */
    double av_photo_residual;
    double av_depth_residual;
    float  av_residual;
    int    residuals_set;
} r360_icp_stats;

void r360_icp_default_params(r360_icp_params* p);

/* alignFrames360(pose_guess, method, occlusion) after setTargetFrame(trg)/setSourceFrame(src)
 * (:4519-4784).  pose_out = getOptimalPose(), H_out = getHessian(), g_out = getGradient().
 * Returns 1 (R360_ILLPOSED) when the reference would print "ILL-POSED" and return early. */
int r360_align360(r360_ctx* ctx, r360_frame* trg, r360_frame* src, const float init[16],
                  int method, int occlusion, const r360_icp_params* p,
                  float pose_out[16], float H_out[36], float g_out[6], r360_icp_stats* st);
int r360_align360_async(r360_ctx* ctx, r360_frame* trg, r360_frame* src, const float init[16],
                        int method, int occlusion, const r360_icp_params* p);
int r360_align360_result(r360_ctx* ctx, float pose_out[16], float H_out[36], float g_out[6],
                         r360_icp_stats* st);

/* Batched alignFrames360 (occlusion 0): n <= R360_MAX_BATCH independent alignments of pairs
 * (trg[j], src[j]) from init[16 j..], each the alignFrames360 of r360_align360 on that pair (same schedule,
 * same per-pair Gauss-Newton state and logic), run as one launch per pass over all pairs.  Batch-invariant:
 * a pair's result is bit-identical in any batch of any size, on any context or rank (the batched grid depends
 * on the level size only).  It equals r360_align360's result to rounding, not bit for bit: a lone alignment
 * sums the same pixels over twice the workgroup records (two per CU) and, on frames with compacted level-0
 * points, with PF 5 instead of PF 6, so a pair whose accept / stop test sits at a rounding edge can stop on
 * another pass (tests/test_gpu_batch_align.py pins the drift).  This is how the reference's callers' many alignFrames360 calls (one per
 * consecutive pair in OdometryRGBD360.cpp:141-257, per keyframe candidate in SphereGraphSLAM /
 * LoopClosure360) fill the GPU.  Frames must share one sphere size and may belong to any ctx of the device:
 * ctx's stream waits for the work already enqueued on their contexts' streams.  _result fills n poses /
 * H / g / stats (NULL skips) and returns the number of ILL-POSED alignments.  One batch per ctx at a time. */
#define R360_MAX_BATCH_ALIGN 16
int r360_align360_batch_async(r360_ctx* ctx, int n, r360_frame* const* trg, r360_frame* const* src,
                              const float* init, int method, const r360_icp_params* p);
int r360_align360_batch_result(r360_ctx* ctx, float* pose_out, float* H_out, float* g_out, r360_icp_stats* st);

/* Dense queue: the alignFrames360 calls of many concurrent registrations (one producer thread per pipeline
 * of frame builds + PbMap stages, e.g. OdometryRGBD360.cpp:141-257 sharded over pipelines) batched on one
 * stream.  A dispatcher thread runs every pending job (up to max_batch of one method / parameter set) as one
 * r360_align360_batch call; the next batch accumulates while one runs.  submit records the frames' build
 * work (their contexts' streams) and returns a ticket at once; collect waits for that job and returns
 * what r360_align360_batch_result returns for the job (0, 1 = ILL-POSED, < 0 error): the batched result,
 * the same in any batch, equal to a lone r360_align360 to rounding (above).  The frames must stay unmodified until
 * their job is collected: a batch waits on each frame's build event, which a rebuild re-records, so a frame
 * rebuilt between submit and dispatch fails the job with an error instead of aligning against the newer build.
 * Every ticket must be collected once.  Thread-safe. */
typedef struct r360_dense_queue r360_dense_queue;
int  r360_dense_queue_create(int device, int max_batch, r360_dense_queue** out);
void r360_dense_queue_destroy(r360_dense_queue* q);
/* the queue's own context (stream, in-kernel span counters, per-launch timing) */
r360_ctx* r360_dense_queue_ctx(r360_dense_queue* q);
int  r360_dense_queue_stats(r360_dense_queue* q, long* batches, long* jobs, int* max_batch_seen);
int  r360_dense_queue_submit(r360_dense_queue* q, r360_frame* trg, r360_frame* src, const float init[16],
                             int method, const r360_icp_params* p, long* ticket);
int  r360_dense_queue_collect(r360_dense_queue* q, long ticket, float pose_out[16], float H_out[36],
                              float g_out[6], r360_icp_stats* st);

/* One fused pass at a fixed pose: errorPhotoICP_sphere (:2545-2739) + calcHessGrad_sphere
 * (:2745-3228) at pyramid level `level`.  H/g in double (sum of the float per-pixel terms). */
int r360_icp_eval(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int level, const float pose[16],
                  int method, const r360_icp_params* p, double H[36], double g[6],
                  double* err2, int* n_valid, int* n_visible);
/* Occlusion-aware pass at `pose` (alignFrames360 occlusion 1 / 2, :4598-4627): H / g of
 * calcHessGrad_sphereOcc{occ} and the value errorPhotoICP_sphereOcc{occ} returns (:3232-3370,
 * :3720-3855); occlusion 0 gives errorPhotoICP_sphere's value.  n_valid = the error's point count
 * (Occ1: photo + depth terms; Occ2: nValidDepthPts), n_visible = the HessGrad's numVisiblePixels. */
int r360_icp_eval_occ(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int level, const float pose[16],
                      int method, int occlusion, const r360_icp_params* p, double H[36], double g[6],
                      double* error, int* n_valid, int* n_visible);

/* ---------------------------------------------------------------- pinhole alignFrames (per sensor)
 * RegisterPhotoICP::alignFrames(pose_guess, method) (:4254-4512) with errorPhotoICP (:560-761) and
 * calcHessGrad (:767-1100), after setTargetFrame / setSourceFrame on sensor k's raw images of two
 * frames (MethodsRegisterRGBD360.cpp:320-345).  Frames need R360_BUILD_SENSOR_PYRAMID.
 * K = {fx, fy, ox, oy} of level 0 (setCameraMatrix); NULL = the calibration's cameraMatrix.
 * Uses p->n_pyr, depth range, std devs and saliency thresholds; the Levenberg-Marquardt constants are
 * alignFrames' own (lambda 0.01, step 10, 10 iterations, tolerances 1e-4).  Returns 1 if ILL-POSED. */
int r360_align_pinhole(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int sensor, const float init[16],
                       int method, const float* K, const r360_icp_params* p, float pose_out[16], float H_out[36],
                       float g_out[6], r360_icp_stats* st);
/* Up to 8 alignments at once (one per listed sensor, init = n x float[16]); _result fills n poses /
 * H / g / stats and returns the number of ILL-POSED jobs. */
int r360_align_pinhole_async(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int n, const int* sensors,
                             const float* init, int method, const float* K, const r360_icp_params* p);
int r360_align_pinhole_result(r360_ctx* ctx, float* poses, float* H, float* g, r360_icp_stats* st);
/* One errorPhotoICP + calcHessGrad pass at `pose` (parity hook): error = avResidual (NaN for
 * PHOTO_CONSISTENCY, as the reference), res = {PhotoResidual, DepthResidual},
 * counts = {nValidPhotoPts, nValidDepthPts, visible}. */
int r360_pinhole_eval(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int sensor, int level, const float pose[16],
                      int method, const float* K, const r360_icp_params* p, double H[36], double g[6],
                      double* error, double res[2], int counts[3]);

/* ---------------------------------------------------------------- RegisterDensePhotoICP (A19)
 * RegisterRGBD360::RegisterDensePhotoICP(frame1, frame2, pose_estim, method, registMode)
 * (RegisterRGBD360.h:344-520): the 8 sensors' pinhole images of frame2 (source) against frame1's
 * (target), Jacobians in the rig frame (calcPhotoICPError_robot, RegisterPhotoICP.h:4905-5076;
 * calcHessianGradient_robot, :5083-5407), sensors summed, LM per level (lambda 1e-3, step 10,
 * tol_residual 0.1).  Frames need R360_BUILD_SENSOR_PYRAMID; p = NULL uses RegisterPhotoICP()'s
 * defaults (4 levels).  As in the reference, the "new" error is evaluated at the unchanged pose, so
 * pose_out = pose_estim and info_out = the Hessian of the last level whose loop ran.
 * Returns 1 (the reference's true) or 0 (ILL-POSED: false, info_out untouched). */
typedef struct {
    double error[8];            /* per level: sum over sensors of calcPhotoICPError_robot   */
    int    ran[8];              /* 1 if the level's LM loop ran (error > tol_residual 0.1)   */
    int    n_visible[8];        /* HessGrad visible pixels per level, 8 sensors             */
    int    n_error[8];          /* error-term visible pixels per level, 8 sensors           */
    int    illposed_level;      /* -1, or the level whose rank test failed                  */
    int    levels;
    int    info_set;            /* 0 if no level ran (the reference's Hessian is then undefined; info = 0) */
    int    pad;
    float  gradient[6];         /* the summed gradient of that level                        */
} r360_dense_stats;
int r360_register_dense(r360_ctx* ctx, r360_frame* frame1, r360_frame* frame2, const float pose_estim[16],
                        int method, int mode, const r360_icp_params* p, float pose_out[16], float info_out[36],
                        r360_dense_stats* st);
/* Parity hook: one level's 8 sensors at `pose`: err[2k] / err[2k+1] = sensor k's photometric / depth
 * part of calcPhotoICPError_robot, H / g = calcHessianGradient_robot's (double sums of the float
 * terms), counts[3k..] = {error visible, error depth terms, HessGrad visible}. */
int r360_dense_robot_eval(r360_ctx* ctx, r360_frame* frame1, r360_frame* frame2, int level, const float pose[16],
                          int method, const r360_icp_params* p, double err[16], double H[8 * 36], double g[8 * 6],
                          int counts[8 * 3]);

/* CPose3D::exp(mu, pseudo) (MRPT; used at RegisterPhotoICP.h:4697). */
void r360_exp_se3(const double mu[6], int pseudo, float T[16]);

/* ---------------------------------------------------------------- PbMap (Frame360 planes)
 * Frame360::getPlanes (Frame360.h:615-640) runs when a frame is built with R360_BUILD_PLANES:
 * cloud + bilateral filter + normals + segmentation on the GPU, per-plane descriptors and the
 * sensor grouping/merging on the host.  One plane = the mrpt::pbmap::Plane fields used on the
 * path, in the rig frame. */
typedef struct {
    float normal[3], center[3], d, area, elongation, curvature, ppal[3], nrgb[3], intensity;
    int   id, sensor, n_inliers, n_hull;
} r360_plane;

int r360_frame_get_planes(r360_frame* f, r360_plane* out, int cap, int* n);
/* Plane::label of plane i (set by the labelization tools, LabelizeFrame360.cpp).  get returns the
 * label length and copies at most cap-1 bytes plus a terminator. */
int r360_frame_set_plane_label(r360_frame* f, int i, const char* label);
int r360_frame_get_plane_label(r360_frame* f, int i, char* buf, int cap);
/* Closed convex hull polygon (polygonContourPtr) of plane i, xyz triples. */
int r360_frame_get_plane_hull(r360_frame* f, int i, float* xyz, int cap, int* n);

/* ---------------------------------------------------------------- keyframe persistence
 * Frame360::sphereCloud (Frame360.h:120): buildSphereCloud's concatenation of the 8 filtered
 * clouds in the rig frame (width = 8*rows/2, height = cols/2), or the cloud set by loadCloud.
 * xyz [cap][3], rgba [cap] (PointXYZRGBA packing b | g<<8 | r<<16 | a<<24); either may be NULL. */
int r360_frame_get_sphere_cloud(r360_frame* f, float* xyz, uint32_t* rgba, size_t cap, int* width, int* height);
/* pcl::io::savePCDFile / PCDReader::read for PointXYZRGBA (Frame360.h:187-193, 326).
 * mode 0 = DATA ascii (the reference's call), 1 = binary, 2 = binary_compressed (LZF). */
int r360_pcd_write(const char* path, const float* xyz, const uint32_t* rgba, int width, int height, int mode);
int r360_pcd_read(const char* path, float* xyz, uint32_t* rgba, size_t cap, size_t* n, int* width, int* height);
int r360_frame_save_cloud(r360_frame* f, const char* path, int mode);
/* loadCloud (Frame360.h:187-193): sets the frame's sphereCloud. */
int r360_frame_load_cloud(r360_frame* f, const char* path);
/* savePlanes / loadPbMap (Frame360.h:195-210, 312-318): gzip file of the frame's PbMap (format in
 * DESIGN.md; MRPT's CSerializable layout is not restated).  A loaded PbMap replaces the frame's
 * planes and registers (r360_register_pbmap) exactly as the one that was saved. */
int r360_frame_save_planes(r360_frame* f, const char* path);
int r360_frame_load_pbmap(r360_frame* f, const char* path);
/* save(path, frame) (Frame360.h:320-330) and load_PbMap_Cloud(path, index) (:222-228):
 * dir/sphereCloud_<i>.pcd + dir/spherePlanes_<i>.pbmap. */
int r360_frame_save(r360_frame* f, const char* dir, unsigned index);
int r360_frame_load_pbmap_cloud(r360_frame* f, const char* dir, unsigned index);

/* ---------------------------------------------------------------- RegisterRGBD360
 * Replaces include/RegisterRGBD360.h:97-337.  registrationType (:260-266). */
enum { R360_DEFAULT_6DoF = 0, R360_PLANAR_3DoF = 1, R360_ODOMETRY_6DoF = 2, R360_PLANAR_ODOMETRY_3DoF = 3 };

/* SubgraphMatcher thresholds: the [global]/[unary]/[binary] keys of the mrpt-pbmap config file that
 * RegisterRGBD360(configFile) loads (RegisterRGBD360.h:97-100, config_files/configLocaliser_*.ini).  A ctx
 * (and each lane of a batch) holds one set; r360_register_pbmap, r360_register* and the batch use it. */
typedef struct {
    int   min_planes_recognition;   /* [global]; RegisterPbMap itself requires 3 matches (:306)            */
    float dist_d;                   /* [unary] plane offset difference (m)                                  */
    float angle;                    /* [unary] normal angle (deg), odometry modes                           */
    float color_threshold;          /* [unary] normalised-rgb difference                                    */
    float intensity_threshold;      /* [unary]                                                              */
    float elongation_threshold;     /* [unary] ratio                                                        */
    float area_threshold;           /* [unary] ratio                                                        */
    float dist_threshold;           /* [binary] centroid-distance ratio                                     */
    float angle_threshold;          /* [binary] relative-normal-angle difference (deg)                      */
    float height_threshold;         /* [binary] relative height of parallel planes (m)                      */
    float cos_angle_parallel;       /* [binary]                                                             */
    float planar_normal_angle;      /* planar modes: vertical-normal tolerance (deg; not an ini key, 10)    */
    long  max_nodes;                /* interpretation-tree node budget: a guard against pathological inputs  */
} r360_match_params;
/* The configLocaliser_sphericalOdometry.ini values (the odometry apps' file). */
void r360_match_params_default(r360_match_params* m);
/* Reads an mrpt-pbmap ini file into m (keys absent from the file keep m's values).  Returns 0, <0 if the
 * file cannot be read. */
int  r360_match_params_load_ini(const char* path, r360_match_params* m);
int  r360_ctx_set_match_params(r360_ctx* ctx, const r360_match_params* m);
int  r360_ctx_get_match_params(const r360_ctx* ctx, r360_match_params* m);
/* The interpretation-tree searches run on ctx (every RegisterPbMap), how many of them stopped at max_nodes, and the
 * most nodes one search visited.  MRPT's SubgraphMatcher (RegisterRGBD360.h:294) searches exhaustively; this one
 * prunes with forward checking (exhaustive result), so a search that reaches the budget is the only way its result
 * can differ from the exhaustive one — and it is counted here, never silent. */
int  r360_ctx_match_stats(r360_ctx* ctx, long* calls, long* truncated, long* max_nodes);
/* That search alone over given tables (host only; the layout r360_pbmap_match_tables returns, areas of the
 * reference planes): best[i] = matched target of reference i or -1.  Returns 1 if max_nodes stopped it, 0 if not. */
int  r360_match_tree_search(int ns, int nt, const uint8_t* unary, const uint64_t* binary, int words,
                            const double* area, long max_nodes, int* best, long* nodes);

/* RegisterPbMap(ref, trg, max_match_planes, mode) (:276-337): returns 1 (good alignment) or 0
 * (insufficient matching / ill-conditioned; pose and info are then left untouched, :306-310).
 * pose = getPose() (target as seen from the reference), info = getInfoMat(), match_pairs =
 * getMatchedPlanes() as (ref id, trg id) pairs, area_matched = getAreaMatched(),
 * area_src/area_trg = the public areaSource/areaTarget members. */
int r360_register_pbmap(r360_ctx* ctx, r360_frame* ref, r360_frame* trg, size_t max_match_planes, int mode,
                        float pose[16], float info[36], int* match_pairs, int pair_cap, int* n_match,
                        float* area_matched, float* area_src, float* area_trg);
/* Register(): RegisterPbMap, then alignFrames360 initialised with rotOffset * P * rotOffset^-1
 * (OdometryKeyFrame360.cpp:167-171, 205, 244-254; guess replaces P when the PbMap registration
 * fails); pose = rotOffset^-1 * getOptimalPose() * rotOffset.  Returns 0, or 1 when the PbMap stage
 * failed and the dense stage started from guess. */
int r360_register(r360_ctx* ctx, r360_frame* ref, r360_frame* trg, const float guess[16],
                  const r360_icp_params* p, size_t max_match_planes, int mode, float pose[16],
                  float info[36], r360_icp_stats* st);
/* Split form for pipelining several pairs: the PbMap stage runs at the call (it waits for the two
 * frames' plane builds), the dense stage is enqueued on ctx's stream; _result waits for it. */
int r360_register_async(r360_ctx* ctx, r360_frame* ref, r360_frame* trg, const float guess[16],
                        const r360_icp_params* p, size_t max_match_planes, int mode);
int r360_register_result(r360_ctx* ctx, float pose[16], float info[36], r360_icp_stats* st);
/* Register() with the dense stage on a dense queue: the PbMap stage runs at the call on ctx (waiting for the
 * frames' plane builds), the rotOffset-conjugated alignFrames360 is submitted to q; collect waits for it and
 * returns what r360_register_result returns. */
int r360_register_submit(r360_ctx* ctx, r360_dense_queue* q, r360_frame* ref, r360_frame* trg, const float guess[16],
                         const r360_icp_params* p, size_t max_match_planes, int mode, long* ticket);
int r360_register_collect(r360_dense_queue* q, long ticket, float pose[16], float info[36], r360_icp_stats* st);

/* OdometryRGBD360 over a frame sequence, pipelined on one GPU (Registration/OdometryRGBD360.cpp:141-257,
 * BASELINE configs[3]; host/sequence.cpp).  Pairs (i, i+1) of [p0, p1) are split into contiguous runs, one per
 * pipeline (a host thread of the object with its own r360_ctx and ring of Frame360 buffers); per pair the new frame
 * is uploaded and built on the GPU and registered with the Register() alias (RegisterPbMap -> rotOffset conjugation
 * -> alignFrames360, OdometryKeyFrame360.cpp:205-254).  With queue > 0 the alignments of all pipelines are batched on
 * one dense queue, `depth` in flight per pipeline, frames built `lookahead` ahead.  Each pair's record equals the
 * single-pair Register() result. */
enum { R360_SEQ_FULL = 0,     /* configs[3]: Register() per pair                                        */
       R360_SEQ_PLANES = 1,   /* configs[1]: planes + RegisterPbMap only                                  */
       R360_SEQ_DENSE = 2 };  /* configs[2] / [4]: stitch + pyramid + alignFrames360 from identity       */
/* One pair record (floats): pose [0,16) column-major in the rig frame of the pair's first frame, PbMap information
 * [16,52), status [52] (0 PbMap good, 1 PbMap failed and the dense stage started from identity, 2 ill-posed), SSO
 * [53], the accepted level-0 error [54], [55] spare. */
#define R360_SEQ_RECORD 56
typedef struct {
    int rows, cols;                 /* per-sensor image size                                            */
    int pipelines;                  /* host threads + streams                                           */
    int queue;                      /* dense queue batch (pairs per launch); 0 = each pipeline aligns alone */
    int depth;                      /* queued: alignments in flight per pipeline                        */
    int lookahead;                  /* queued: frames built ahead of the pair in hand                   */
    int plane_batch;                /* plane stages of up to this many frames per launch on one stream (0: each
                                       pipeline builds its frames' planes on its own stream)            */
    int workload;                   /* R360_SEQ_*                                                       */
    size_t max_match_planes;        /* RegisterPbMap (25)                                               */
    int mode;                       /* registrationType (PLANAR_3DoF)                                   */
    r360_icp_params icp;            /* alignFrames360 (nPyr 5, stdDevPhoto 3/255, 20 level-0 iterations) */
} r360_sequence_params;
typedef struct r360_sequence r360_sequence;
void r360_sequence_default_params(r360_sequence_params* p);
/* extrinsics_dir: Rt_0{1..8}.txt (NULL / "" = the shipped calibration) */
int  r360_sequence_create(int device, const r360_sequence_params* p, const char* extrinsics_dir, r360_sequence** out);
void r360_sequence_destroy(r360_sequence* s);
/* Registers pairs [p0, p1) `repeats` times.  Frame i's raw images (BGR u8 8 x rows x cols x 3, depth u16 mm
 * 8 x rows x cols) are bgr[i - p0] / depth[i - p0] for i in [p0, p1]: host memory (page-locked for asynchronous
 * uploads) or, with device_inputs, device memory.  The repeats x (p1 - p0) registrations form one stream (repeat-
 * major) cut into P contiguous pieces, one per pipeline; runs (optional): n_runs (first, last + 1) pairs tiling
 * [p0, p1) in order, pipeline k taking run k of every repeat instead.  records: repeats x (p1 - p0) x
 * R360_SEQ_RECORD floats.  Returns 0, or < 0 with the failing pipeline's error. */
int  r360_sequence_run(r360_sequence* s, int p0, int p1, const void* const* bgr, const void* const* depth,
                       int device_inputs, int repeats, const int* runs, int n_runs, float* records);
/* Pipelines and the dense queue (NULL when unqueued). */
int  r360_sequence_info(r360_sequence* s, int* pipelines, r360_dense_queue** queue);
/* The plane queue's batches, frames and largest batch so far, and its context (NULL without one). */
int  r360_sequence_plane_stats(r360_sequence* s, long* batches, long* frames, int* max_batch_seen, r360_ctx** ctx);
/* Pipeline p's context, calibration, frame ring (up to cap handles) and OS thread id. */
int  r360_sequence_pipeline(r360_sequence* s, int p, r360_ctx** ctx, r360_calib** calib, r360_frame** frames, int cap,
                            int* n_frames, long* thread_id);
/* Host seconds per pipeline since the last reset: out[8 p + k], k = 0 load + build enqueue (with the collects that
 * free a buffer), 1 PbMap stage (RegisterPbMap and submit), 2 dense wait, 3 pairs registered; within 0: 4 build
 * enqueue, 5 upload enqueue, 6 (queued) collects before a buffer refill; 7 unused. */
int  r360_sequence_host_times(r360_sequence* s, double* out, int reset);
/* Parity hook: the two raster sweeps of OrganizedMultiPlaneSegmentation::refine as k_refine* run them, on
 * 8 sensors' refinement states (-1 no label, -2 non-planar label, m >= 0 planar model m) and closeness
 * masks (bit m: the pixel is within 0.02 of model m), w x h each; rb = -1: the wavefront sweeps (the
 * default path: 64-row bands pipelined through LDS for h <= 512), -2: the wavefront with a workgroup barrier
 * per diagonal, 0: one wave per sensor walks all rows, rb > 0: rb rows per band.  out = the swept states.
 * Returns the number of sensors whose wavefront second sweep needed corrections of the flat-index wrap push
 * (re-runs or the single-wave fallback; rb < 0), else 0; < 0 on error. */
int r360_refine_eval(const int8_t* state, const uint64_t* mask, int w, int h, int rb, int8_t* out);
/* SubgraphMatcher constraint tables (k_match_tables): unary [ns][nt], binary [(i*nt+j)][words]
 * bitsets over (k*nt+l).  Returns words.  Inspection/parity hook. */
int r360_pbmap_match_tables(r360_ctx* ctx, r360_frame* ref, r360_frame* trg, size_t max_match_planes,
                            int mode, int* ns, int* nt, int* sid, int* tid, uint8_t* unary,
                            uint64_t* binary, int cap);

/* ---------------------------------------------------------------- batched registrations (§8f-4)
 * Many independent pair registrations on one GPU, as SphereGraphSLAM's tracking loop
 * (SLAM/SphereGraphSLAM.cpp:169-231: RegisterPbMap against up to numCheckRegistration = 5 previous
 * keyframes) and LoopClosure360's candidate checks (include/LoopClosure360.h:280-366: RegisterPbMap
 * PLANAR_3DoF, gate on matches/area, alignFrames360 refinement) issue them.  A batch owns `lanes`
 * worker contexts (own HIP stream, ICP state and matcher scratch) and runs the jobs of one call
 * concurrently, one host thread per lane.  Every job is the sequential call itself on its lane's
 * context: the result of a batched job is identical to r360_register_pbmap / r360_align360 on the
 * same frames (lone alignments, not the batched grid of r360_align360_batch).  Frames may belong to any ctx of the same device; each lane's stream waits for
 * the frames' build work before reading them.  The caller must not modify or destroy a frame while a
 * batch call that names it runs.  Calls on one batch are serialised: a call made while another thread's
 * call runs waits for it. */
typedef struct r360_batch r360_batch;
int  r360_batch_create(int device, int lanes, r360_batch** out);
void r360_batch_destroy(r360_batch* b);
int  r360_batch_lanes(const r360_batch* b);
/* The matcher thresholds of every lane (r360_ctx_set_match_params). */
int  r360_batch_set_match_params(r360_batch* b, const r360_match_params* m);

/* dense stage of one job */
enum {
    R360_JOB_PBMAP_ONLY = 0,  /* RegisterPbMap only (SphereGraphSLAM tracking)                          */
    R360_JOB_GATED = 1,       /* alignFrames360 only when RegisterPbMap succeeded with n_match > min_matches
                                 and area_matched > min_area (LoopClosure360.h:298, 342)                */
    R360_JOB_ALWAYS = 2       /* Register(): alignFrames360 from the PbMap pose, or from `guess` when the
                                 PbMap stage failed (OdometryKeyFrame360.cpp:205-254)                   */
};
typedef struct {
    r360_frame* ref;          /* RegisterPbMap(ref, trg, ...): pRef360 (RegisterRGBD360.h:276)           */
    r360_frame* trg;
    int   dense;              /* R360_JOB_*                                                               */
    int   ref_is_source;      /* dense roles. 0: setTargetFrame(ref), setSourceFrame(trg)
                                 (OdometryKeyFrame360.cpp:248-249, LoopClosure360.h:348-349).
                                 1: setSourceFrame(ref), setTargetFrame(trg) (LoopClosure360.h:309-310) */
    float guess[16];          /* R360_JOB_ALWAYS fallback pose (rig frame)                               */
} r360_pair_job;
typedef struct {
    int   good;               /* RegisterPbMap's return value (1 / 0)                                    */
    int   n_match;            /* getMatchedPlanes().size()                                               */
    float area_matched, area_src, area_trg, sso_pbmap;   /* getAreaMatched(), areaSource, areaTarget,
                                 areaMatched / areaSource (SphereGraphSLAM.cpp:214-215; 0 if not good)   */
    float pbmap_pose[16];     /* getPose() (identity if not good)                                        */
    float pbmap_info[36];     /* getInfoMat() (zeros if not good)                                        */
    int   dense_rc;           /* -1: dense stage not run; 0 ok; 1 ill-posed (R360_ILLPOSED)               */
    float pose[16];           /* rotOffset^-1 * getOptimalPose() * rotOffset (LoopClosure360.h:313, 352) */
    float hessian[36];        /* getHessian()                                                            */
    r360_icp_stats stats;     /* SSO, accepted error, iterations                                         */
} r360_pair_result;

/* Runs the n jobs.  max_match_planes/mode apply to every RegisterPbMap; min_matches/min_area gate
 * R360_JOB_GATED jobs; p = the dense stage's RegisterPhotoICP parameters (PHOTO_DEPTH, occlusion 0).
 * Returns 0, or the first job error (< 0, message in r360_last_error()). */
int r360_batch_register(r360_batch* b, const r360_pair_job* jobs, int n, size_t max_match_planes, int mode,
                        int min_matches, float min_area, const r360_icp_params* p, r360_pair_result* out);

/* SphereGraphSLAM tracking step (SphereGraphSLAM.cpp:169-231): RegisterPbMap(kfs[j], frame,
 * max_match_planes, mode) for j = n_kf-1, n_kf-2, ... (newest keyframe first) while fewer than
 * num_check candidates and fewer than no_assoc_threshold failures were tried; the first good one wins.
 * All candidates are registered at once; *chosen = index into kfs of the winner, or -1 ("No
 * registration available").  result (optional) = the winner's r360_pair_result; cand (optional,
 * min(n_kf, num_check, no_assoc_threshold) entries) = every candidate's result in reference order. */
int r360_track_frame(r360_batch* b, r360_frame* const* kfs, int n_kf, r360_frame* frame, int num_check,
                     int no_assoc_threshold, size_t max_match_planes, int mode, int* chosen,
                     r360_pair_result* result, r360_pair_result* cand);

/* Inspection hooks of the per-pixel plane half (parity tests).  Sizes: 8 x (rows/2) x (cols/2). */
typedef struct {
    int   label, count, start_idx, n_contour, n_fit;
    float centroid[3], cov[9], model[4], curvature;
} r360_region;
int r360_frame_get_cloud(r360_frame* f, float* xyz4, uint8_t* rgb4, float* nrm4, float* dist);
int r360_frame_get_labels(r360_frame* f, int* lab, int* labf);
int r360_frame_get_regions(r360_frame* f, int sensor, r360_region* out, int cap, int* n);

/* ---------------------------------------------------------------- multi-GPU sequence driver (§8(e))
 * Pairs of a sequence shard one contiguous run per GPU (one process per GPU); the per-pair records
 * {pose, information, status, ...} are all-gathered to every rank over RCCL (xGMI) and rank 0 composes the
 * trajectory (Registration/OdometryRGBD360.cpp:257).  Rank 0 creates the id; the caller distributes it.
 * Host buffers in and out; each call returns when its result is on the host. */
typedef struct r360_comm r360_comm;
int  r360_comm_unique_id(uint8_t id[128]);
int  r360_comm_init(int device, int nranks, int rank, const uint8_t id[128], r360_comm** out);
void r360_comm_destroy(r360_comm* c);
/* recv[r * bytes .. (r + 1) * bytes) = rank r's send (ncclAllGather). */
int  r360_comm_allgather(r360_comm* c, const void* send, void* recv, size_t bytes);
/* v[i] = max over the ranks of v[i] (ncclAllReduce / ncclMax, f64). */
int  r360_comm_allreduce_max(r360_comm* c, double* v, int n);

/* Plain device buffers (inputs kept resident in HBM, r360_frame_upload_device).  kind: 0 host->device,
 * 1 device->host, 2 device->device; synchronous. */
int  r360_dev_alloc(int device, size_t bytes, void** out);
int  r360_dev_free(void* p);
int  r360_dev_copy(void* dst, const void* src, size_t bytes, int kind);

/* ---------------------------------------------------------------- synthetic scenes
 * Procedural indoor room rendered by the 8 rig cameras.  Deterministic in
 * (seed, frame).  Rig pose of frame `frame` along the generator's planar path; pose_out
 * (column-major) is that rig pose in the room frame. */
int r360_synth_frame(const r360_calib* calib, uint32_t seed, const float rig_pose[16],
                     uint8_t* bgr8, uint16_t* depth8);
/* Host-only variant (no GPU needed): rt8 = the 8 extrinsics Rt_k, column-major, back to back. */
int r360_synth_frame_rt(int rows, int cols, const float* rt8, uint32_t seed, const float rig_pose[16],
                        uint8_t* bgr8, uint16_t* depth8);
int r360_synth_path_pose(uint32_t seed, int frame, float pose_out[16]);

/* ---------------------------------------------------------------- test hooks
 * The float asinf/atan2f program used by the projection (libm_f32.h, bit-identical to x86-64 glibc)
 * evaluated on the host (on_device = 0) or on the GPU (on_device = 1). */
/* The ICP pass's fast-guarded vs the exact spherical projection of points (X, Y, Z) for an
 * nRows x nCols sphere: pixel-decision mismatches (must be 0) and deferred (exact) lanes.  _pose:
 * LUT points (lx, ly, lz) transformed by pose (col-major 4x4) first, fast and exact transforms. */
int r360_proj_check(const float* X, const float* Y, const float* Z, int n, int nRows, int nCols,
                    unsigned long long* mismatches, unsigned long long* fallbacks);
int r360_proj_check_pose(const float* lx, const float* ly, const float* lz, int n, const float pose[16], int nRows,
                         int nCols, unsigned long long* mismatches, unsigned long long* fallbacks);
/* sqrt_rn / div_rn (the pass's correctly rounded f32 sqrt / division) against the compiler's IEEE
 * operations on n hashed operands: out = {sqrt mismatches, division mismatches}, both must be 0. */
int r360_rn_check(unsigned n, unsigned seed, unsigned long long out[2]);
/* The device ILL-POSED test: Eigen FullPivLU<Matrix<float,6,6>>::rank() of n row-major matrices. */
int r360_rank6(const float* M, int n, int* ranks);
/* The device GN solve x = -H^-1 g (RegisterPhotoICP.h:4693; Gaussian elimination with partial pivoting in
 * double) of n systems: H row-major n x 36, g n x 6, x n x 6. */
int r360_solve6(const double* H, const double* g, int n, double* x);
int r360_libm_eval(const float* x, const float* y, const float* z, int n, float* asin_out, float* atan2_out,
                   int on_device);

/* s_memrealtime stamps (100 MHz) of the last ICP pass; written only by a -DR360_STAMPS build. */
int r360_ctx_debug_stamps(r360_ctx* ctx, unsigned long long* out12);

/* Lone alignFrames360 (r360_align360*, occlusion 0) as ONE launch per pyramid level (k_icp_level: the level's passes
 * in a persistent grid, the step's workgroup handing each pass over to the others) instead of one launch per pass.
 * Same grid, records and steps: results are bit-identical either way (st->persistent says which ran).  Off by
 * default: measured slower on MI355X.  Used only when every level's grid fits one resident
 * round and no other persistent alignment of the process is in flight. */
int r360_ctx_persistent_levels(r360_ctx* ctx, int enable);

/* Latency mode (no reference counterpart: a scheduling choice; on by default).  On: a thread waiting for the PbMap of
 * a frame built on ctx polls the frame's GPU part itself and runs its assembly tasks; r360_frame_upload_async copies
 * the depth images first and the BGR images on a second stream beside the plane stage's geometric part; a lone
 * frame's plane stage is replayed as two graphs.  Off: waits sleep on the assembly pool, both copies and every
 * launch go in the ctx stream's order (what a context among many pipelines wants: the sequence runner turns it off
 * for more than one pipeline).  Results are the same either way, bit for bit. */
int r360_ctx_latency_mode(r360_ctx* ctx, int enable);

/* ---------------------------------------------------------------- timing hooks (bench) */
/* enable: 0 off, 1 every launch on ctx's stream, 2 the level-0 ICP passes only (HIP events around each) */
int r360_ctx_timing(r360_ctx* ctx, int enable);
/* Per-kernel accumulated device time (ms) and launch counts since the last reset. */
int r360_ctx_timing_read(r360_ctx* ctx, const char* kernel, double* ms, long* launches);
int r360_ctx_timing_reset(r360_ctx* ctx);
/* In-kernel execution spans of the fused ICP passes at one pyramid level (earliest workgroup start to
 * the end of the last workgroup, s_memrealtime), summed in microseconds, and the pass count, since the
 * last reset.  Unlike stream events they exclude queueing behind other streams' kernels. */
int r360_ctx_kernel_time(r360_ctx* ctx, int level, double* us_sum, long* passes);
/* the same, plus the job passes those launches ran (a batched launch runs one per pair; NULL skips) */
int r360_ctx_kernel_stats(r360_ctx* ctx, int level, double* us_sum, long* launches, long* job_passes);
/* Profiling: host time of the ctx's RegisterPbMap calls: out[0] s waiting for the frames' PbMaps (GPU plane
 * stage + host assembly), out[1] s in the match tables, out[2] s in the interpretation tree + ConsistencyTest,
 * out[3] calls; out[4] s of PbMap assembly (the frames' host threads), out[5] frames; reset != 0 zeroes them.
 * (No reference counterpart: instrumentation of r360_register_pbmap and the frames' assembly.) */
int r360_ctx_host_times(r360_ctx* ctx, double out[6], int reset);
int r360_ctx_kernel_time_reset(r360_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
