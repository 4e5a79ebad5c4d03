// r360_internal.h — internal types shared by the HIP kernels and the host runtime of
// librgbd360_hip.so.  Not part of the ABI.
#pragma once
#include <atomic>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <memory>
#include <string>
#include <thread>
#include <vector>
#include "../../include/rgbd360_hip.h"

#define R360_PI 3.14159265359  // include/Miscellaneous.h:44 (double literal)

// Experiment knobs (pass forms, grid caps, CU masks, priorities, A/B switches) read the environment only in the
// experiment builds (make exp / stamps, -DR360_EXPERIMENTS=1, lib/librgbd360_hip_exp.so): in the product library
// R360_KNOB is its default and the variable's name is not even in the binary, so no environment variable can
// change a registration.
#ifndef R360_EXPERIMENTS
#define R360_EXPERIMENTS 0
#endif
#if R360_EXPERIMENTS
#include <cstdlib>
#define R360_KNOB(name, dflt) (std::getenv(name) ? std::atoi(std::getenv(name)) : (dflt))
#define R360_KNOB_STR(name) (std::getenv(name))
#else
#define R360_KNOB(name, dflt) (dflt)
#define R360_KNOB_STR(name) ((const char*)nullptr)
#endif

// ------------------------------------------------------------------ error plumbing
void r360_set_error(const char* fmt, ...);
#define R360_HIP(call)                                                                  \
    do {                                                                                \
        hipError_t _e = (call);                                                         \
        if (_e != hipSuccess) {                                                         \
            r360_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(_e)); \
            return -1;                                                                  \
        }                                                                               \
    } while (0)

// Binds the calling thread to `device` (HIP's current device is per host thread): every entry point that enqueues
// work or creates streams / events calls it first, so contexts of any device can be driven from any thread (the
// pipelines' pool threads of a rank with LOCAL_RANK >= 1 never call hipSetDevice themselves).
inline int bind_device(int device) {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != device) R360_HIP(hipSetDevice(device));
    return 0;
}

// argument check of a C-ABI entry point: sets the thread's error and returns -2
#define CHECK_ARG(cond, msg)                 \
    do {                                     \
        if (!(cond)) {                       \
            r360_set_error("%s", msg);       \
            return -2;                       \
        }                                    \
    } while (0)

// ------------------------------------------------------------------ device layouts
// One pyramid level of a frame's sphere, as the fused ICP pass reads it:
//   p0[i] = {gray, depth}          (source stream AND target gather)   8 B/px
//   tg[i] = {gx, gy, dgx, dgy}     (target gradients, seam-masked)    16 B/px
struct LevelBufs {
    int rows = 0, cols = 0;
    float2* p0 = nullptr;
    float4* tg = nullptr;
    // the level's valid source pixels (minDepth < depth < maxDepth, RegisterPhotoICP.h:4578) in raster
    // order as {LUT_xyz_sphere point (:4580-4582), gray}: the ICP pass streams these instead of the image
    // (launch_pyramid builds them; the count is the frame's d_npts[level])
    float4* pts = nullptr;
    // level 0 only: the level's {gray, depth} as the stitch produced them, 4 B per pixel: range in mm (u16) |
    // luma (u8) << 16.  gray = luma * (float)(1/255), depth = range * 0.001f reproduce p0 bit for bit; the
    // level-0 ICP pass (PF 6) streams the source and gathers the target {gray, depth} from these.
    uint32_t* pk = nullptr;
};
constexpr int R360_SRC_BLOCK = 4096;   // pixels per block of the source-point compaction
// one level's inputs / output of the compaction (a device-side table per frame, fixed at creation)
struct SrcLevel { const float2* p0; float4* pts; const float* sinphi; const float* cosphi; const float* sinth;
                  const float* costh; int rows, cols; };

// Per-geometry trigonometric tables, computed on the host with the same float expressions
// as the reference (RegisterPhotoICP.h:4555-4569), so the device LUT is bit-identical.
struct LevelTrig {
    float* sinphi = nullptr;  // [rows]
    float* cosphi = nullptr;  // [rows]
    float* sinth = nullptr;   // [cols]
    float* costh = nullptr;   // [cols]
};

struct IcpConst {
    float min_d, max_d, sd_photo, sd_depth, thr_int, thr_depth;
    float sd_photo_inv_f;     // float stdDevPhoto_inv = 1./stdDevPhoto   (:2774)
    float pad0;
    double sd_photo_inv_d;    // double stdDevPhoto_inv = 1./stdDevPhoto  (:2561)
    double tol_res, tol_upd, lambda;
    int max_iters, fixed_iters0, n_pixels, level;
    int occ;                  // alignFrames360 occlusion: 0 plain, 1 Occ1, 2 Occ2 (:4598-4627)
    unsigned seq;             // ICP pass: launch sequence number on the ctx (never 0), the record flags' value
};

// Device-resident Gauss-Newton state of one alignFrames360 call.
struct alignas(16) IcpState {
    float pose[16];     // pose_estim
    float cand[16];     // pose evaluated by the next pass
    float Hcur[36];     // H at pose_estim
    float gcur[6];
    float Hout[36];     // 'hessian' member: H of the last solve
    float gout[6];
    float upd[6];
    float sso_cur, sso;
    double error, diff_error;
    int it, loops, evals, active, stop, illposed, passes, level;
    int iters[8], evals_l[8];
    unsigned ticket;
    int pad1;
    double lm_lambda;   // alignFrames (pinhole) Levenberg-Marquardt lambda (:4301)
    int lm_phase;       // 0: the pending candidate is the undamped step, 1: the LM retry (:4381-4412)
    int pad2;
    double gn_lambda;   // alignFrames360 lambda of the current level: 1 at the level start, /= 5 per accepted update
    double pad3;
    // the residual members the error functions assign (RegisterPhotoICP.h:183-189): of the last evaluated
    // pass (av_*) and, for alignFrames, the copies taken at each loop iteration's start (av_*_t, :4329-4332)
    double av_photo, av_depth, av_photo_t, av_depth_t;
    float av_res, av_res_t;
    int av_set;         // bit 0 photo/depth of the last pass assigned, bit 1 av_res assigned, bits 2/3 the copies
    double sums[32];    // last pass sums (eval mode)
    unsigned long long dbg[12];  // s_memrealtime stamps of the diagnostic build (-DR360_STAMPS)
    // last 16 B, never written back by a persistent level launch's step: set by a workgroup whose wait for a
    // pass's step timed out (the launch then ends and the alignment reports an error)
    int fault;
    int pad4[3];
};

// One alignment of a batched ICP launch (blockIdx.y = job): the pair's level buffers and its own GN state,
// record area, arrival counters and deferred-pixel queue.  A single alignment is a batch of one.
constexpr int R360_MAX_BATCH = R360_MAX_BATCH_ALIGN;
struct IcpJob {
    const float2* src;          // source level {gray, depth}
    const float2* trg;          // target level {gray, depth}
    const float4* tg;           // target level gradients
    const float4* pts;          // source level compacted points (PF 4 / 5)
    const int* npts;            // their count
    const uint32_t* spk;        // level 0: source packed {range mm, luma} image (PF 6)
    const uint32_t* tpk;        // level 0: target packed image
    IcpState* S;
    double* partials;           // per-workgroup records
    unsigned* gcnt;             // per-workgroup record flags (R360_POLL) / group arrival counters (16384 words)
    int* dq;                    // deferred-pixel queues
};
struct IcpJobs { IcpJob j[R360_MAX_BATCH]; };   // passed by value (kernel arguments, 1152 B)

constexpr int R360_KT_SLOTS = 26;
#ifndef R360_GROUP_SUM   // 1: group records summed by each ticket group's last workgroup; 0 (experiment builds): flat sum
#define R360_GROUP_SUM 1
#endif
#ifndef R360_POLL   // 0: arrival tickets; 1 (experiment builds): record flags polled by the job's last workgroup
#define R360_POLL 0
#endif
#ifndef R360_TICKET_GROUPS_N   // experiment builds may regroup the same 16384 counter words
#define R360_TICKET_GROUPS_N 16
#endif
constexpr int R360_TICKET_GROUPS = R360_TICKET_GROUPS_N;
constexpr int R360_TICKET_STRIDE = 16384 / R360_TICKET_GROUPS_N;   // uints between group counters (4 KB at 16)
// the persistent level launch's pass generation word: the last of the 16384 counter words, never a group counter
constexpr int R360_PERSIST_FLAG_WORD = 16383;
static_assert(R360_TICKET_STRIDE > 1, "the generation word must not be a group counter");

// Pass sums.  Occlusion variants: NVALID counts photo terms (Occ1) or accepted points (Occ2), NDEPTH
// the depth terms (Occ1), ERR2 the photometric and ERR2D the depth squared residuals.
enum { R360_SUM_NVALID = 27, R360_SUM_NVIS = 28, R360_SUM_NDEPTH = 29, R360_SUM_ERR2D = 30, R360_SUM_ERR2 = 31,
       R360_NSUMS = 32 };

// ------------------------------------------------------------------ plane half
#include "plane_math.h"
#define R360_MAX_MODELS 64     // planar models per sensor (refinement closeness bit masks are 64-bit)
#define R360_MAX_BIG 512       // labels with > 80 points per sensor
#define R360_REFINE_BANDS 64   // row bands per sensor of the banded refinement sweeps

// One planar model of segment() (PlanarRegion statistics + ModelCoefficients)
struct PlaneModel {
    int label, n_fit;
    int big;                 // index of the label in the sensor's large-label list
    float v[4];
    float centroid[3];
    float cov[9];
    float curvature;
};

// Per-model device output copied to the host for the PbMap descriptors
struct alignas(16) PlaneOut {
    r360p::Moments stats;   // final inliers: rig-frame moments + colour sums
    PlaneModel model;
    int start;              // inlier_indices[i][0]
    int n_contour, n_vox, vox_fill;
    int hull_n;             // the region's hull candidates (k_hullpre: contour or voxel points not strictly inside
                            // the Akl-Toussaint octagon), at contour_off / vox_off of the pinned pools
    float bmin[3], bmax[3]; // local-frame bounds of the inliers (VoxelGrid)
    long contour_off, vox_off;
};

// (region, voxel) hash cell of the VoxelGrid fallback and its compacted output
struct VoxCell {
    unsigned long long tag;  // 0 = empty; ((sensor*64 + model + 1) << 48) | voxel index
    double s[3];
    unsigned cnt, pad;
};
struct VoxOut {
    long long key;
    float x, y, z, pad;
};

// Global accumulators of the refined regions' grouped-moment kernel (plane_seg.hip): exact moments in the rig frame +
// colour sums and local-frame bounds, in R360_GM_COPIES copies.
#define R360_GM_COPIES 8
struct RegionPart {
    r360p::Moments m;
    float bmin[3], bmax[3];
};

// Device buffers of a frame's plane half (allocated on the first CLOUD/PLANES build)
struct PlaneBufs {
    int w = 0, h = 0;
    float4* cloud = nullptr;    // [8][h][w] {x, y, z, 0}
    uchar4* rgb = nullptr;      // [8][h][w] {r, g, b, 0}
    float4* nrm = nullptr;      // [8][h][w] {nx, ny, nz, d = p.n}
    float* dist0 = nullptr;     // distance-map init (depth-change map)
    float* dist = nullptr;      // distance map
    float2* grids = nullptr;    // bilateral grids, 8 x 2 x grid_cells
    long grid_cells = 0;
    int sd_max = 0;
    int* zmm = nullptr;         // per-sensor depth range for the bilateral grid: [8] min, [8] max (ordered ints)
    int* parent = nullptr;      // union-find parents, then root ranks
    int* root = nullptr;
    int* lab = nullptr;         // CCL labels (per-sensor ids, -1 none)
    int* labf = nullptr;        // labels after refinement
    int* cnt = nullptr;         // label sizes [8][N]
    int* aux = nullptr;         // the large labels' first pixels [8][R360_MAX_BIG] (plane_seg.hip)
    int* chunk = nullptr;       // per-chunk counts of the numbering kernels [8][ceil(N / 256)]
    int* nlab = nullptr;        // [8]
    int* big = nullptr;         // [8][R360_MAX_BIG]
    int* nbig = nullptr;        // [8]
    r360p::Moments* mom = nullptr;   // [8][R360_MAX_BIG] the large labels' moments
    PlaneModel* models = nullptr;    // [8][R360_MAX_MODELS]
    int* nmodels = nullptr;          // [8]
    int8_t* state = nullptr;         // refinement state [8][N]
    int8_t* state2 = nullptr;        // refinement state after the first sweep [8][N]
    int8_t* rbnd = nullptr;          // banded refinement: each band's assignments into the next band's first row
    int* rflag = nullptr;            //   [8][R360_REFINE_BANDS][w] and whether they changed that row [8][..]
    unsigned long long* mask = nullptr;  // closeness masks [8][N]
    uint16_t* rcode = nullptr;           // wavefront refinement, skewed [8][h + w - 1][h]: state | push conditions
    unsigned long long* rmsk = nullptr;  //   closeness masks, skewed
    int8_t* rf1 = nullptr;               //   first sweep's states, skewed
    int8_t* rf2 = nullptr;               //   second sweep's states, skewed
    PlaneOut* out = nullptr;         // [8][R360_MAX_MODELS]
    RegionPart* gpart = nullptr;     // [R360_GM_COPIES][8][R360_MAX_MODELS] region accumulators (k_gm<true>)
    float4* contour = nullptr;       // contour points kept by the hull prefilter (pinned host)
    long contour_cap = 0;
    VoxOut* vox = nullptr;           // voxel-fallback centroids kept by the hull prefilter (pinned host)
    float4* contour_dev = nullptr;   // the traced contours (device; k_trace -> k_hullpre)
    VoxOut* vox_dev = nullptr;       // all voxel-fallback centroids (device; k_vox_compact -> k_hullpre)
    long vox_cap = 0;
    long* totals = nullptr;          // [2] pool usage
    int* err = nullptr;              // error bits
    // pinned host mirrors
    PlaneOut* h_out = nullptr;
    int* h_nmodels = nullptr;        // [8], then err at [8], totals at (long*)(h_nmodels + 10)
    // host assembly thread (planes_enqueue -> planes_finish)
    hipEvent_t done = nullptr;
    hipEvent_t ready = nullptr;      // plane queue: recorded on the frame's stream once its inputs are built
    std::shared_ptr<struct PlaneTicket> ticket;   // plane queue: set when the batch's kernels and `done` are enqueued
    bool asm_busy = false;           // the host assembly is queued or running (host/pbmap.cpp AsmPool; under its lock)
    int worker_rc = 0;
    std::string worker_err;
};
struct PbMapHost;                    // host PbMap (host/pbmap.cpp)

// One frame's plane-stage buffers as the plane kernels see them.  Every plane kernel takes a PlaneBatch (by value, in
// the kernel-argument segment) and serves frame blockIdx.z of it (k_normals*: blockIdx.z / 8), so one launch runs
// the same stage of up to R360_PLANE_BATCH frames of the same size (host/plane_queue.cpp), and a lone frame's build
// is a batch of one.
struct PlaneDev {
    const float* depth_m; const uint8_t* bgr;
    float4* cloud; uchar4* rgb; float4* nrm; float* dist0; float* dist; float2* grids; int* zmm;
    int* parent; int* root; int* lab; int* labf; int* cnt; int* aux; int* chunk; int* nlab; int* big; int* nbig;
    r360p::Moments* mom; PlaneModel* models; int* nmodels;
    int8_t* state; int8_t* state2; unsigned long long* mask; int8_t* rbnd; int* rflag;
    uint16_t* rcode; unsigned long long* rmsk; int8_t* rf1; int8_t* rf2;
    PlaneOut* out; RegionPart* gpart; float4* contour; float4* contour_dev; VoxOut* vox; VoxOut* vox_dev; long* totals; int* err;
    PlaneOut* h_out; int* h_nmodels; const float* rt;
    VoxCell* vhash; int* vlist; int* vcnt;
    long contour_cap, vox_cap;
    unsigned long long vhash_cap;
};
#define R360_PLANE_BATCH 8
struct PlaneBatch { PlaneDev f[R360_PLANE_BATCH]; };
static_assert(sizeof(PlaneBatch) + 256 <= 4096, "the plane batch travels as a kernel argument");

// ------------------------------------------------------------------ host objects
struct r360_plane_queue;
struct VoxSlot;
struct r360_ctx {
    r360_plane_queue* plane_q = nullptr;   // frames built on this ctx run their plane stage on this queue (batched)
    int device = 0;
    hipStream_t stream = nullptr;
    bool stream_borrowed = false;   // another object's stream (a pipeline sharing its dense queue's): not destroyed
    hipEvent_t wait_ev = nullptr;   // blocking-sync event: host waits sleep instead of spinning
    // RegisterPbMap's match tables run on the device's shared high-priority match stream (pbmap.cpp): on the
    // ctx's stream they would queue behind the new frame's stitch and pyramid, which the host does not need yet
    hipStream_t mstream = nullptr;
    hipEvent_t mwait_ev = nullptr;
    // host time of the ctx's RegisterPbMap calls (ns): 0 waiting for the frames' PbMaps (GPU plane stage + host
    // assembly), 1 match tables (upload, kernel, wait), 2 interpretation tree + ConsistencyTest, 3 calls; of its
    // frames' assembly threads: 4 PbMap assembly after the GPU part, 5 frames
    std::atomic<long long> host_ns[6] = {};
    IcpState* d_state = nullptr;
    double* d_partials = nullptr;
    unsigned* d_gticket = nullptr;   // group arrival counters of the ICP pass (R360_TICKET_GROUPS x 4 KB)
    int* d_defer = nullptr;          // ICP pass (PF 3): per-wave queues of deferred (exactly re-projected) pixels
    long defer_cap = 0;
    // in-kernel execution spans of the ICP passes (s_memrealtime, 100 MHz): [0] earliest workgroup start
    // of the running pass, [1+l] summed spans at level l, [9+l] pass counts, [17] job arrivals of the running
    // pass (low 32 bits: jobs arrived, high: jobs that ran; the last arrival closes the span), [18+l] job
    // passes run at level l (a batched launch runs one per pair); R360_KT_SLOTS entries
    unsigned long long* d_ktime = nullptr;
    // occlusion variants: per-source target pixel / exact inverse range / flags, per-target counts,
    // offsets (exclusive scan) and the grouped source lists (icp_kernels.hip, k_occ_*)
    long occ_cap = 0;
    int* occ_tgt = nullptr;
    float* occ_dinv = nullptr;
    uint8_t* occ_flags = nullptr;
    int* occ_cnt = nullptr;
    int* occ_off = nullptr;
    int* occ_list = nullptr;
    int* occ_bsum = nullptr;
    int partials_cap = 0;
    unsigned icp_seq = 0;            // ICP launches on this ctx (IcpConst::seq)
    // alignFrames360's fixed pass sequence (levels n_pyr-1..0, every GN pass) captured once per pair of frame
    // buffers and replayed as one graph launch (r360_align360_async): the key lists every pointer, size and
    // parameter the launches read, so a replay issues exactly the launches the loop would
    struct AlignGraph { std::vector<uintptr_t> key; hipGraphExec_t exec = nullptr; unsigned long long used = 0; };
    std::vector<AlignGraph> graphs;
    unsigned long long graph_clock = 0;
    // graphs are captured on a stream of their own (capture_stream) and launched on `stream`: an event recorded on a
    // stream that is capturing cannot be queried meanwhile, and the assembly pool polls events recorded on `stream`
    hipStream_t cap_stream = nullptr;
    // a lone frame's plane stage (split_upload contexts) replayed as two graphs, the geometric part and the model part
    // (the BGR wait between them), keyed by the frame's plane buffers and geometry (pbmap.cpp plane_graph_launch)
    struct PlaneGraph { std::string key; hipGraphExec_t exec = nullptr; unsigned long long used = 0; };
    std::vector<PlaneGraph> plane_graphs;
    IcpState* h_state = nullptr;  // pinned
    int timing = 0;
    r360_ctx* stats_sibling = nullptr;   // a dense queue's second stream: its kernel statistics are reported with these
    int persist_levels = 0; // r360_ctx_persistent_levels: lone alignments as one launch per level
    int persist_held = 0;   // this ctx holds the process's persistent-launch slot (runtime.cpp, persist_slot)
    int async_persist = 0;  // the pending r360_align360 runs as persistent level launches
    // a thread that waits for the PbMap of a frame built on this ctx polls the frame's GPU part itself and runs its
    // assembly tasks (pbmap.cpp planes_join): the latency of a lone frame.  The queued sequence runner turns it off
    // for its pipelines (their waits would spin host cores the other pipelines' frames need)
    bool join_help = true;
    // with split_upload (the same latency-bound callers) r360_frame_upload_async copies the depth images first on the
    // ctx stream and the BGR images after them on up_stream, beside the plane stage's geometric part, which needs only
    // the depth; the stage waits for the BGR images (f->bgr_ev) just before its colour moments
    bool split_upload = true;
    hipStream_t up_stream = nullptr;
    hipEvent_t up_ev = nullptr;
    std::vector<hipEvent_t> ev_pool;
    int ev_used = 0;
    struct TimedLaunch { std::string name; int a, b; };
    std::vector<TimedLaunch> pending;
    struct Acc { double ms = 0; long n = 0; };
    std::vector<std::pair<std::string, Acc>> acc;
    // async-align bookkeeping
    int async_nL = 0, async_pending = 0;
    double align_t0 = 0, align_est = 0;   // the pending lone alignment's enqueue time, the previous one's duration (s)
    // batched alignFrames360 (r360_align360_batch_*): per-job state / records / counters / queues
    int batch_cap = 0;               // jobs the batch buffers hold
    long bdefer_cap = 0;             // deferred-queue entries per job
    IcpState* d_bstate = nullptr;
    double* d_bpartials = nullptr;   // [batch_cap][partials_cap][32]
    unsigned* d_bgticket = nullptr;  // [batch_cap][R360_TICKET_GROUPS * R360_TICKET_STRIDE]
    int* d_bdefer = nullptr;         // [batch_cap][bdefer_cap]
    IcpState* h_bstate = nullptr;    // pinned
    int batch_n = 0, batch_pending = 0;
    std::vector<hipEvent_t> sync_ev; // producer-stream events the batch waits on
    // pinhole alignFrames (pinhole_kernels.hip): one state and one record area per job (sensor)
    IcpState* d_pin_state = nullptr;
    double* d_pin_partials = nullptr;
    IcpState* h_pin_state = nullptr;   // pinned
    int pin_pending = 0;
    // RegisterDensePhotoICP (robot_kernels.hip): job table, per-job records / sums / tickets, result
    struct RobotJob* d_rob_jobs = nullptr;
    struct RobotJob* h_rob_jobs = nullptr;     // pinned
    double* d_rob_partials = nullptr;
    double* d_rob_sums = nullptr;
    double* h_rob_sums = nullptr;              // pinned
    unsigned* d_rob_tickets = nullptr;
    struct RobotOut* d_rob_out = nullptr;
    struct RobotOut* h_rob_out = nullptr;      // pinned
    // PbMap matcher scratch (k_match_tables)
    int match_cap = 0;                       // planes per subgraph
    r360_match_params match{};               // SubgraphMatcher thresholds (r360_ctx_set_match_params)
    // interpretation-tree searches on this ctx, those cut by the node budget, and the most nodes one search visited
    std::atomic<long> match_calls{0}, match_truncated{0}, match_nodes_max{0};
    float* d_match_desc = nullptr;
    uint8_t* d_unary = nullptr;
    unsigned long long* d_bin = nullptr;
    uint8_t* h_unary = nullptr;              // pinned
    unsigned long long* h_bin = nullptr;     // pinned
    // VoxelGrid hash table (plane builds of the frames on this ctx)
    VoxCell* d_vhash = nullptr;
    long vhash_cap = 0;
    int* d_vlist = nullptr;          // cells each k_vox_hash workgroup claimed [vlist_cap], its count per workgroup
    int* d_vcnt = nullptr;           //   [vcnt_cap] (k_vox_compact walks these instead of the whole table)
    long vlist_cap = 0, vcnt_cap = 0;
    // r360_frames_build: voxel scratch of batch slots 1.. (slot 0 is the table above); VoxSlot is declared below
    std::vector<VoxSlot> bvox;
    // Register() in flight (r360_register_async)
    int reg_pending = 0, reg_good = 0;
    float reg_info[36];
};

struct ClamsDev {
    int width = 0, height = 0, bin_w = 0, bin_h = 0, nx = 0, ny = 0, num_bins = 0;
    double bin_depth = 2.0;
    float* d_mult = nullptr;    // [8][ny*nx][num_bins]
    float* d_counts = nullptr;  // [8][ny*nx][num_bins]
};

struct r360_calib {
    r360_ctx* ctx = nullptr;
    int rows = 0, cols = 0;
    float rt[8][16];       // Rt_  (col-major)
    float rt_inv[8][16];   // Rt_inv
    float K[9];            // cameraMatrix (col-major)
    bool has_intrinsics = false;
    ClamsDev clams;
    // stitch tables (Frame360.h:1104-1129): per sphere row sin/cos(phi_i); per col sin/cos(theta_i)
    int sph_rows = 0, sph_cols = 0;
    float* d_st_sinphi = nullptr;
    float* d_st_cosphi = nullptr;
    float* d_st_sinth = nullptr;
    float* d_st_costh = nullptr;
    float* d_rt_inv = nullptr;  // [8][16]
    float* d_rt = nullptr;      // [8][16]
    // ICP trig tables per pyramid level of the sphere
    int n_levels = 0;
    LevelTrig trig[R360_MAX_PYR];
};

// Host copy of Frame360::sphereCloud as loadCloud leaves it (io.cpp)
struct SphereCloudHost {
    int width = 0, height = 0;
    std::vector<float> xyz;      // [n][3]
    std::vector<uint32_t> rgba;  // PCL PointXYZRGBA packing: b | g<<8 | r<<16 | a<<24
};

struct r360_frame {
    r360_ctx* ctx = nullptr;
    const r360_calib* calib = nullptr;
    int rows = 0, cols = 0, sph_rows = 0, sph_cols = 0, n_levels = 0;
    uint8_t* d_bgr = nullptr;      // [8][rows][cols][3]
    // bgr_split: the last write of d_bgr was a split upload's copy on the ctx's upload stream (r360_ctx::split_upload),
    // recorded on bgr_ev; its readers (the stitch, the sensor pyramid, the plane stage's colours) and the next writer
    // wait on bgr_ev.  Otherwise d_bgr is written in the ctx stream's order and nothing waits (bgr_wait: nullptr)
    hipEvent_t bgr_ev = nullptr;
    bool bgr_split = false;
    hipEvent_t bgr_wait() const { return bgr_split ? bgr_ev : nullptr; }
    uint16_t* d_depth = nullptr;   // [8][rows][cols] mm
    float* d_depth_m = nullptr;    // [8][rows][cols] undistorted metres
    int* d_npts = nullptr;         // [R360_MAX_PYR] valid source points per level (LevelBufs::pts)
    int* d_src_cnt = nullptr;      // [R360_MAX_PYR][blocks] compaction scratch
    SrcLevel* d_src_levels = nullptr;  // [n_levels]
    int src_blocks = 0;
    uint8_t* d_sph_bgr = nullptr;  // [H][W][3]
    uint16_t* d_sph_depth = nullptr;
    LevelBufs lv[R360_MAX_PYR];
    // per-sensor pinhole pyramids (R360_BUILD_SENSOR_PYRAMID): level l = [8][rows>>l][cols>>l], no seam mask
    LevelBufs sp[R360_MAX_PYR];
    int n_slevels = 0;
    // R360_BUILD_* stages done (atomic: a frame built on one thread may have its sphere built from another,
    // while the first reads its plane flags)
    std::atomic<unsigned> built{0};
    PlaneBufs pl;
    PbMapHost* pbmap = nullptr;
    uint64_t timestamp = 0;            // Frame360::timeStamp (Frame360.h:181-184)
    unsigned compacted = 0;            // bit l: lv[l].pts / d_npts[l] hold level l's compacted source points
    // the pyramid build compacts every level: a lone alignment's passes (PF 5) read the compacted points.  Frames that
    // only enter batched alignments (compact_all unset: the sequence runner's queued ring) skip it on every level a
    // batched pass streams as an image (PF 6 at level 0, PF 8 above; round 6: two launches per frame fewer)
    bool compact_all = true;
    SphereCloudHost* sphere_cloud = nullptr;  // sphereCloud set by loadCloud (Frame360.h:187-193)
    // builds recorded on the frame's build event (runtime.cpp frame_build_event_record): a dense-queue job snapshots
    // it at submit and its batch refuses to run if the frame was rebuilt meanwhile (the event would then stand for
    // the newer build)
    std::atomic<unsigned> build_gen{0};
};

// ------------------------------------------------------------------ kernel launchers
hipStream_t capture_stream(r360_ctx* ctx);   // ctx->cap_stream, created on first use (nullptr on failure)
int launch_undistort(r360_frame* f);
int launch_stitch(r360_frame* f);
int launch_pyramid(r360_frame* f);
int launch_src_compaction(r360_frame* f, unsigned levels);   // compacted source points of the levels (bit l)
constexpr int R360_CU_MASK_WORDS = 8;
bool r360_cu_mask(int device, int for_queue, uint32_t* mask);   // CU partition experiment (runtime.cpp)
int launch_sphere_level0(r360_frame* f);   // level 0 {gray, depth m} from the frame's sphere images
int launch_sensor_pyramid(r360_frame* f);
// pinhole alignFrames: intrinsics of level 0 (setCameraMatrix) and the jobs of one batched launch
struct PinJobs { int sensor[8]; int n; };
constexpr int R360_PIN_MAX_BLOCKS = 256;   // workgroups per job and pass (record area per job)
int launch_pin_level(r360_ctx* ctx, const r360_frame* trg, const r360_frame* src, int level, int method,
                     const IcpConst& C, const float K[4], const PinJobs& J, int first, int eval_only);
// RegisterDensePhotoICP (A19): one job = (pyramid level, sensor); matrices col-major
struct RobotJob {
    const float2* src;        // source sensor level {gray, depth}
    const float2* trg;        // target sensor level {gray, depth}
    const float4* tg;         // target gradients {gx, gy, dgx, dgy}
    int rows, cols;
    float fx, fy, ox, oy, inv_fx, inv_fy;          // calcPhotoICPError_robot's float intrinsics
    double fxd, fyd, oxd, oyd, inv_fxd, inv_fyd;   // calcHessianGradient_robot's double intrinsics
    float Mrel[16];           // relPoseCam = Rt^-1 * pose * Rt (float products)
    float Rt[16], P[16], Rti[16];
};
constexpr int R360_ROBOT_MAX_JOBS = 8 * R360_MAX_PYR;
constexpr int R360_ROBOT_MAX_BLOCKS = 256;
constexpr int TPB_ROBOT = 256;   // k_robot_pass workgroup size
struct RobotGrid { int block0[R360_ROBOT_MAX_JOBS + 1]; int njobs; };
struct RobotOut {
    float info[36], grad[6];
    double error[8];
    int ran[8], n_visible[8], n_error[8];
    int ok, illposed_level, any, pad;
};
int launch_robot(r360_ctx* ctx, const RobotJob* d_jobs, const RobotGrid& grid, int method, const IcpConst& C,
                 int finalize_levels);
int launch_icp_level(r360_ctx* ctx, const r360_frame* trg, const r360_frame* src, int level,
                     int method, const IcpConst& C, int first, int eval_only);
// One pass over n jobs at pyramid level `level` (plain alignFrames360 only: C.occ == 0); the jobs' frames
// share the level geometry of `geom`.  kt: the ctx's in-kernel span counters.
int launch_icp_jobs(r360_ctx* ctx, const IcpJobs& jobs, int n, const r360_frame* geom, int level, int method,
                    const IcpConst& C, int first, int eval_only);
int icp_blocks_for(int n_pixels);
// The persistent level launch (k_icp_level): all `passes` passes of a plain (C.occ == 0) lone alignment's level in
// one launch.  icp_level_persist_ok: whether level's pass grid fits one resident round of that kernel with a
// workgroup per CU to spare (and the build has it); launch_icp_level_persist enqueues it.
bool icp_level_persist_ok(r360_ctx* ctx, const r360_frame* src, int level, int method);
// a coarse level of a batch as one persistent launch (k_icp_levels_batch); 1 = no such form for it (launch per pass)
int launch_icp_levels_batch(r360_ctx* ctx, const IcpJobs& jobs, int n, const r360_frame* geom, int level, int method,
                            const IcpConst& C, int passes);
int launch_icp_level_persist(r360_ctx* ctx, const r360_frame* trg, const r360_frame* src, int level, int method,
                             const IcpConst& C, int passes);
// sizes ctx->d_defer for passes over up to n_pixels pixels (synchronises the ctx stream when it grows,
// so it never frees a queue an enqueued pass still uses); call before enqueuing a level sequence
int ensure_defer(r360_ctx* ctx, long n_pixels);
// sizes ctx's batch buffers for n jobs over frames of up to n_pixels level-0 pixels (synchronises when growing)
int ensure_batch(r360_ctx* ctx, int n, long n_pixels);
// ctx's stream waits for the work enqueued so far on the streams of the frames' contexts
int ctx_wait_frames(r360_ctx* ctx, r360_frame* const* frames, int n);
// The plane stage of a batch of F frames of the same size (PlaneBatch, r360_internal.h) on stream st; tctx: the
// context whose per-launch timing (r360_ctx_timing) records the launches, if any
struct PlaneGeom { int rows, cols, w, h, sd_max; long grid_cells; };
PlaneGeom plane_geom(const r360_frame* f);
int launch_cloud_normals(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st, r360_ctx* tctx);
// bgr_ev: the F frames' BGR events (nullptr: none), waited on before the colour moments (launch_rgb, k_gm<true>)
int launch_segmentation(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st, r360_ctx* tctx,
                        const hipEvent_t* bgr_ev);
int launch_rgb(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st);   // the clouds' colours (P.rgb)
int launch_segmentation_geom(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st, r360_ctx* tctx);
int launch_segmentation_model(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st, r360_ctx* tctx);
int launch_plane_publish(const PlaneBatch& B, int F, hipStream_t st);   // plane outputs -> pinned host buffers
// voxel-fallback scratch the plane stage of one frame uses (its context's, or a plane queue slot's)
struct VoxScratch { VoxCell* vhash; unsigned long long cap; int* vlist; int* vcnt; };
// the voxel scratch sizes a frame of G needs: hash cells, list entries, list groups (workgroups)
void vox_scratch_need(const PlaneGeom& G, long* cells, long* entries, long* groups);
// one batch slot's voxel scratch with its capacities (plane queue slots, r360_frames_build slots)
struct VoxSlot { VoxScratch v{nullptr, 0, nullptr, nullptr}; long cells = 0, entries = 0, groups = 0; };
int vox_slot_reserve(VoxSlot& s, const PlaneGeom& G, hipStream_t st);   // zeroed hash (memset on st when it grows)
void vox_slot_free(VoxSlot& s);
PlaneDev plane_dev(const r360_frame* f, const VoxScratch& vs);
int plane_bufs_alloc(r360_frame* f);
void plane_bufs_free(r360_frame* f);
int planes_enqueue(r360_frame* f);
int planes_spawn_assembly(r360_frame* f);
// Plane queue (host/plane_queue.cpp): the plane stage of frames built on any context attached to it (ctx->plane_q),
// batched into launches over up to max_batch frames on the queue's own stream
int plane_queue_create(int device, int max_batch, r360_plane_queue** out);
void plane_queue_destroy(r360_plane_queue* q);
int plane_queue_submit(r360_plane_queue* q, r360_frame* f);   // after plane_bufs_alloc; records f's ready event
int plane_queue_stats(const r360_plane_queue* q, long* batches, long* frames, int* max_batch_seen);
r360_ctx* plane_queue_ctx(r360_plane_queue* q);
int ctx_vhash_reserve(r360_ctx* ctx, long min_cells, long list_entries, long list_groups);
int planes_finish(r360_frame* f);
// plane queue ticket: 1 the frame's batch and `done` event are enqueued, 0 not yet, -1 the batch failed (*err)
int plane_ticket_poll(const std::shared_ptr<struct PlaneTicket>& tk, std::string* err);
// rotOffset (157.5 deg about x, OdometryRGBD360.cpp:138-139) and its inverse; column-major 4x4 product C = A*B
void r360_rot_offset(float Ro[16], float Ri[16]);
void r360_mul4(const float* A, const float* B, float* C);
int planes_assemble(r360_frame* f);
void planes_join(r360_frame* f);

// timing helpers (host_runtime.cpp)
int  timing_begin(r360_ctx* ctx, const char* name);
// Wait for everything enqueued on the context's stream, sleeping (blocking-sync event) rather than
// spinning, so many pipelines' host threads can wait while plane assembly threads keep the cores.
int  ctx_wait(r360_ctx* ctx);
// waits for a recorded event, polling it with short sleeps (no core spins for the wait)
int  event_wait(hipEvent_t e);
void timing_end(r360_ctx* ctx, int slot);
