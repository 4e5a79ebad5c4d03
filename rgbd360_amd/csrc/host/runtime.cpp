// runtime.cpp — host side of librgbd360_hip.so: contexts, Calib360, Frame360 and the
// RegisterPhotoICP::alignFrames360 driver.  Everything here is plumbing around the HIP kernels
// (frame_kernels.hip, icp_kernels.hip); the per-pixel work never runs on the CPU.
#include <atomic>
#include <chrono>
#include <dlfcn.h>
#include <mutex>
#include <unordered_map>
#include <sys/prctl.h>
#include <cmath>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../r360_internal.h"

static thread_local std::string g_err;
void r360_set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}
extern "C" const char* r360_last_error(void) { return g_err.c_str(); }
extern "C" const char* r360_version(void) { return "rgbd360_amd 0.1 (gfx950)"; }

// The shipped data directory (calibration, matcher ini files, samples): $R360_DATA_DIR, else data/ of the tree the
// library was built in (<tree>/rgbd360_amd/lib/librgbd360_hip.so -> <tree>/data).  The reference's callers rely on
// PROJECT_SOURCE_PATH for the same files (Calib360.h:107, :125; OdometryRGBD360.cpp:68).
extern "C" const char* r360_data_dir(void) {
    static const std::string dir = [] {
        if (const char* e = getenv("R360_DATA_DIR")) return std::string(e);
        Dl_info info;
        if (dladdr((void*)&r360_data_dir, &info) && info.dli_fname) {
            std::string p(info.dli_fname);
            for (int up = 0; up < 3; ++up) {            // strip the file name, lib/, rgbd360_amd/
                const size_t s = p.find_last_of('/');
                p = s == std::string::npos ? std::string(".") : p.substr(0, s);
            }
            return p + "/data";
        }
        return std::string("data");
    }();
    return dir.c_str();
}

// dir, or the shipped calibration's sub-directory where dir is NULL / "" (the reference's "" default argument)
static std::string calib_dir_or_default(const char* dir, const char* sub) {
    if (dir && *dir) return dir;
    return std::string(r360_data_dir()) + "/calib/" + sub;
}


// ------------------------------------------------------------------ timing (HIP events on the ctx stream)
// Waits for a recorded event by polling it with short sleeps.  hipEventSynchronize spins a core for the
// whole wait even on a blocking-sync event (measured: every per-frame assembly thread and pipeline thread
// of the bench burned its wait, 15 of 16 host cores at 16 pipelines), and a sleeping poll gives the cores
// back to the PbMap host stages; the added latency is at most one sleep (<= 100 us) on ms-scale waits.
// Polls e with short sleeps.  While it sleeps, the waiting thread's timer slack is 1 us (its own setting, per
// thread): with Linux's default 50 us slack a 20 us sleep overslept to ~70 us, so every short wait (a lone
// alignment's result, RegisterPbMap's match tables) paid up to that much after the GPU had finished.  The caller's
// own slack is restored before returning (the thread may be the application's).
namespace {
// 1 us timer slack on the calling thread for the duration of a wait (restored after): the default 50 us made every
// short sleep of a poll loop overshoot
struct Slack {
    long old;
    Slack() : old(prctl(PR_GET_TIMERSLACK, 0UL, 0UL, 0UL, 0UL)) {
        if (old != 1000) (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
    }
    ~Slack() {
        if (old > 0 && old != 1000) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)old, 0UL, 0UL, 0UL);
    }
};
double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
}  // namespace

int event_wait(hipEvent_t e) {
    const hipError_t r0 = hipEventQuery(e);
    if (r0 == hipSuccess) return 0;
    if (r0 != hipErrorNotReady) {
        r360_set_error("hipEventQuery -> %s", hipGetErrorString(r0));
        return -1;
    }
    Slack slack;
    for (int k = 0;; ++k) {
        std::this_thread::sleep_for(std::chrono::microseconds(k < 32 ? 5 : k < 96 ? 20 : 100));
        const hipError_t r = hipEventQuery(e);
        if (r == hipSuccess) return 0;
        if (r != hipErrorNotReady) {
            r360_set_error("hipEventQuery -> %s", hipGetErrorString(r));
            return -1;
        }
    }
}

int ctx_wait(r360_ctx* ctx) {
    R360_HIP(hipEventRecord(ctx->wait_ev, ctx->stream));
    return event_wait(ctx->wait_ev);
}

// A lone alignment's result wait.  The previous alignment on the ctx took align_est seconds from its enqueue: until
// 90 % of that has passed the wait checks every 50 us, then every ~2 us for at most 200 us, then as event_wait (whose
// 20 us polls by then came ~10 us late on average).  A wrong estimate (another frame size) costs at most one coarse
// check.  *waited: the alignment was still running at the first check, so the time to the end of this wait measures
// the alignment; a result call that came after it had finished says nothing about its duration (a late
// caller inflated the next estimate and with it the fine-poll window).
static int align_wait(r360_ctx* ctx, bool* waited) {
    R360_HIP(hipEventRecord(ctx->wait_ev, ctx->stream));
    *waited = false;
    const hipError_t r0 = hipEventQuery(ctx->wait_ev);
    if (r0 == hipSuccess) return 0;
    if (r0 != hipErrorNotReady) {
        r360_set_error("hipEventQuery -> %s", hipGetErrorString(r0));
        return -1;
    }
    *waited = true;
    const double est = ctx->align_est;
    if (est > 0 && est < 0.05) {
        Slack slack;
        const double t_fine = ctx->align_t0 + 0.9 * est, t_end = t_fine + std::min(2.1 * est, 200e-6);
        for (;;) {
            const double t = now_s();
            if (t > t_end) break;
            const double left = t_fine - t;
            std::this_thread::sleep_for(std::chrono::microseconds(left > 50e-6 ? 50 : left > 2e-6 ? (long)(left * 1e6) : 2));
            const hipError_t r = hipEventQuery(ctx->wait_ev);
            if (r == hipSuccess) return 0;
            if (r != hipErrorNotReady) {
                r360_set_error("hipEventQuery -> %s", hipGetErrorString(r));
                return -1;
            }
        }
    }
    return event_wait(ctx->wait_ev);
}

int timing_begin(r360_ctx* ctx, const char* name) {
    if (!ctx || !ctx->timing) return -1;
    if (ctx->timing == 2 && strcmp(name, "k_icp_pass_L0") != 0) return -1;   // level-0 passes only
    if (ctx->ev_used + 2 > (int)ctx->ev_pool.size()) {
        for (int i = 0; i < 64; ++i) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return -1;
            ctx->ev_pool.push_back(e);
        }
    }
    const int a = ctx->ev_used++, b = ctx->ev_used++;
    hipEventRecord(ctx->ev_pool[a], ctx->stream);
    ctx->pending.push_back({name, a, b});
    return (int)ctx->pending.size() - 1;
}
void timing_end(r360_ctx* ctx, int slot) {
    if (slot < 0 || !ctx) return;
    hipEventRecord(ctx->ev_pool[ctx->pending[slot].b], ctx->stream);
}
static void timing_flush(r360_ctx* ctx) {
    if (!ctx->timing || ctx->pending.empty()) return;
    hipStreamSynchronize(ctx->stream);
    for (auto& p : ctx->pending) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, ctx->ev_pool[p.a], ctx->ev_pool[p.b]);
        bool found = false;
        for (auto& kv : ctx->acc)
            if (kv.first == p.name) { kv.second.ms += ms; kv.second.n += 1; found = true; break; }
        if (!found) { r360_ctx::Acc a; a.ms = ms; a.n = 1; ctx->acc.push_back({p.name, a}); }
    }
    ctx->pending.clear();
    ctx->ev_used = 0;
}

extern "C" int r360_ctx_persistent_levels(r360_ctx* ctx, int enable) {
    CHECK_ARG(ctx, "null ctx");
    ctx->persist_levels = enable ? 1 : 0;
    return 0;
}

hipStream_t capture_stream(r360_ctx* ctx) {
    if (!ctx->cap_stream && hipStreamCreateWithFlags(&ctx->cap_stream, hipStreamNonBlocking) != hipSuccess) {
        ctx->cap_stream = nullptr;
        r360_set_error("hipStreamCreateWithFlags failed (graph capture stream)");
    }
    return ctx->cap_stream;
}

extern "C" int r360_ctx_latency_mode(r360_ctx* ctx, int enable) {
    CHECK_ARG(ctx, "null ctx");
    ctx->join_help = enable != 0;
    ctx->split_upload = enable != 0;
    return 0;
}

extern "C" int r360_ctx_timing(r360_ctx* ctx, int enable) {
    CHECK_ARG(ctx, "null ctx");
    timing_flush(ctx);
    ctx->timing = enable;
    return 0;
}
extern "C" int r360_ctx_timing_read(r360_ctx* ctx, const char* kernel, double* ms, long* launches) {
    CHECK_ARG(ctx && kernel, "null arg");
    timing_flush(ctx);
    *ms = 0; *launches = 0;
    for (auto& kv : ctx->acc)
        if (kv.first == kernel) { *ms = kv.second.ms; *launches = kv.second.n; }
    return 0;
}
extern "C" int r360_ctx_timing_reset(r360_ctx* ctx) {
    CHECK_ARG(ctx, "null ctx");
    timing_flush(ctx);
    ctx->acc.clear();
    return 0;
}

// ------------------------------------------------------------------ context
// CU partition experiment (off by default).  R360_QUEUE_CU_EXCL=n keeps n CUs out of the dense queue's stream
// (R360_QUEUE_CU_PAT=spread: every (CUs / n)-th CU, =high: the last n); R360_PIPE_CU=excl puts every other context's
// stream on exactly those n CUs.  Returns true and fills mask when the stream of that kind gets a CU mask.
bool r360_cu_mask(int device, int for_queue, uint32_t* mask) {
    static const int excl = R360_KNOB("R360_QUEUE_CU_EXCL", 0);
    static const bool high = R360_KNOB_STR("R360_QUEUE_CU_PAT") && strcmp(R360_KNOB_STR("R360_QUEUE_CU_PAT"), "high") == 0;
    static const bool pipe = R360_KNOB_STR("R360_PIPE_CU") && strcmp(R360_KNOB_STR("R360_PIPE_CU"), "excl") == 0;
    if (excl <= 0 || (!for_queue && !pipe)) return false;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= excl ||
        cus > 32 * R360_CU_MASK_WORDS)
        return false;
    for (int w = 0; w < R360_CU_MASK_WORDS; ++w) mask[w] = 0;
    const int step = cus / excl;
    for (int i = 0; i < cus; ++i) {
        const bool ex = high ? i >= cus - excl : (i % step == step - 1 && i / step < excl);
        if (ex != (bool)for_queue) mask[i / 32] |= 1u << (i % 32);
    }
    return true;
}

extern "C" int r360_ctx_create(int device, r360_ctx** out) {
    CHECK_ARG(out, "null out");
    int n = 0;
    R360_HIP(hipGetDeviceCount(&n));
    CHECK_ARG(device >= 0 && device < n, "invalid device ordinal");
    R360_HIP(hipSetDevice(device));
    r360_ctx* c = new r360_ctx;
    c->device = device;
    // R360_CTX_PRIORITY=1: contexts' streams at the device's highest priority (the dense queue keeps the normal
    // one, r360_dense_queue_create); an experiment knob, off by default
    static const int ctx_prio = R360_KNOB("R360_CTX_PRIORITY", 0);
    uint32_t mask[R360_CU_MASK_WORDS];
    if (ctx_prio) {
        int least = 0, greatest = 0;
        R360_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        R360_HIP(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest));
    } else if (r360_cu_mask(device, 0, mask)) {   // R360_PIPE_CU=excl: contexts on the dense queue's excluded CUs
        R360_HIP(hipExtStreamCreateWithCUMask(&c->stream, R360_CU_MASK_WORDS * 32, mask));
    } else {
        R360_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    }
    R360_HIP(hipEventCreateWithFlags(&c->wait_ev, hipEventDisableTiming | hipEventBlockingSync));
    // Initial contents on the ctx's own stream: hipMemset runs on the null stream, which does not order with a
    // non-blocking stream (and returns before it completes), so a first kernel on c->stream could overtake it.
    R360_HIP(hipMalloc(&c->d_state, sizeof(IcpState)));
    R360_HIP(hipMemsetAsync(c->d_state, 0, sizeof(IcpState), c->stream));
    c->partials_cap = 2048;
    R360_HIP(hipMalloc(&c->d_partials, sizeof(double) * 32 * c->partials_cap));
    R360_HIP(hipMalloc(&c->d_gticket, sizeof(unsigned) * R360_TICKET_STRIDE * R360_TICKET_GROUPS));
    R360_HIP(hipMemsetAsync(c->d_gticket, 0, sizeof(unsigned) * R360_TICKET_STRIDE * R360_TICKET_GROUPS, c->stream));
    R360_HIP(hipMalloc(&c->d_ktime, sizeof(unsigned long long) * R360_KT_SLOTS));
    R360_HIP(hipMemsetAsync(c->d_ktime, 0, sizeof(unsigned long long) * R360_KT_SLOTS, c->stream));
    R360_HIP(hipMemsetAsync(c->d_ktime, 0xff, sizeof(unsigned long long), c->stream));
    R360_HIP(hipHostMalloc(&c->h_state, sizeof(IcpState), hipHostMallocDefault));
    r360_match_params_default(&c->match);
    *out = c;
    return 0;
}

void persist_release(r360_ctx* ctx);

extern "C" void r360_ctx_destroy(r360_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    persist_release(c);
    for (auto e : c->ev_pool) hipEventDestroy(e);
    hipEventDestroy(c->wait_ev);
    if (c->mwait_ev) hipEventDestroy(c->mwait_ev);   // mstream is the device's shared match stream
    for (auto& g : c->graphs) hipGraphExecDestroy(g.exec);
    for (auto& g : c->plane_graphs) hipGraphExecDestroy(g.exec);
    if (c->cap_stream) hipStreamDestroy(c->cap_stream);
    hipFree(c->d_state);
    hipFree(c->d_partials);
    hipFree(c->d_gticket);
    hipFree(c->d_defer);
    hipFree(c->d_ktime);
    hipHostFree(c->h_state);
    hipFree(c->d_bstate); hipFree(c->d_bpartials); hipFree(c->d_bgticket); hipFree(c->d_bdefer);
    hipHostFree(c->h_bstate);
    for (auto e : c->sync_ev) hipEventDestroy(e);
    hipFree(c->d_pin_state); hipFree(c->d_pin_partials); hipHostFree(c->h_pin_state);
    hipFree(c->d_rob_jobs); hipFree(c->d_rob_partials); hipFree(c->d_rob_sums); hipFree(c->d_rob_tickets);
    hipFree(c->d_rob_out); hipHostFree(c->h_rob_jobs); hipHostFree(c->h_rob_sums); hipHostFree(c->h_rob_out);
    hipFree(c->d_match_desc); hipFree(c->d_unary); hipFree(c->d_bin); hipFree(c->d_vhash);
    hipFree(c->d_vlist); hipFree(c->d_vcnt);
    for (auto& s : c->bvox) vox_slot_free(s);
    hipHostFree(c->h_unary); hipHostFree(c->h_bin);
    if (c->up_stream) {
        hipStreamSynchronize(c->up_stream);
        hipStreamDestroy(c->up_stream);
        hipEventDestroy(c->up_ev);
    }
    if (!c->stream_borrowed) hipStreamDestroy(c->stream);
    delete c;
}

extern "C" int r360_ctx_kernel_stats(r360_ctx* ctx, int level, double* us_sum, long* launches, long* job_passes) {
    CHECK_ARG(ctx && level >= 0 && level < 8 && us_sum && launches, "invalid arguments");
    *us_sum = 0.0;
    *launches = 0;
    if (job_passes) *job_passes = 0;
    for (r360_ctx* c = ctx; c; c = (c == ctx) ? ctx->stats_sibling : nullptr) {
        unsigned long long k[R360_KT_SLOTS];
        if (ctx_wait(c)) return -1;
        R360_HIP(hipMemcpy(k, c->d_ktime, sizeof k, hipMemcpyDeviceToHost));
        *us_sum += (double)k[1 + level] * 0.01;   // 100 MHz ticks
        *launches += (long)k[9 + level];
        if (job_passes) *job_passes += (long)k[18 + level];
    }
    return 0;
}

extern "C" int r360_ctx_kernel_time(r360_ctx* ctx, int level, double* us_sum, long* passes) {
    return r360_ctx_kernel_stats(ctx, level, us_sum, passes, nullptr);
}

// Host time of the ctx's RegisterPbMap calls (profiling): out[0..2] seconds waiting for the frames' PbMaps,
// in the match tables, in the tree search + ConsistencyTest; out[3] calls; out[4] seconds of PbMap assembly of
// the ctx's frames, out[5] frames.  reset != 0 zeroes the counters.
extern "C" int r360_ctx_host_times(r360_ctx* ctx, double out[6], int reset) {
    CHECK_ARG(ctx && out, "null arg");
    for (int k = 0; k < 6; ++k) {
        const long long v = reset ? ctx->host_ns[k].exchange(0) : ctx->host_ns[k].load();
        out[k] = (k == 3 || k == 5) ? (double)v : (double)v * 1e-9;
    }
    return 0;
}

extern "C" int r360_ctx_kernel_time_reset(r360_ctx* ctx) {
    CHECK_ARG(ctx, "null ctx");
    for (r360_ctx* c = ctx; c; c = (c == ctx) ? ctx->stats_sibling : nullptr) {
        if (ctx_wait(c)) return -1;
        R360_HIP(hipMemsetAsync(c->d_ktime, 0, sizeof(unsigned long long) * R360_KT_SLOTS, c->stream));
        R360_HIP(hipMemsetAsync(c->d_ktime, 0xff, sizeof(unsigned long long), c->stream));
    }
    return 0;
}

extern "C" int r360_ctx_sync(r360_ctx* c) {
    CHECK_ARG(c, "null ctx");
    return ctx_wait(c);
}
extern "C" void* r360_ctx_stream(r360_ctx* c) { return c ? (void*)c->stream : nullptr; }

// ------------------------------------------------------------------ Calib360
static void inverse4(const float* T, float* Ti) {  // rigid-or-general 4x4 inverse in double
    double m[16], inv[16];
    for (int i = 0; i < 16; ++i) m[i] = T[i];
    inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    for (int i = 0; i < 16; ++i) Ti[i] = (float)(inv[i] / det);
}

static int upload_floats(float** dptr, const std::vector<float>& h) {
    if (*dptr) hipFree(*dptr);
    R360_HIP(hipMalloc(dptr, sizeof(float) * (h.size() ? h.size() : 1)));
    R360_HIP(hipMemcpy(*dptr, h.data(), sizeof(float) * h.size(), hipMemcpyHostToDevice));
    return 0;
}

// Trigonometric tables with the reference's exact float expressions:
//   stitchImage (Frame360.h:1104-1129) and the alignFrames360 LUT (RegisterPhotoICP.h:4555-4569).
// sph_rows / sph_cols: the sphere size; 0 = the one stitchSphericalImage produces from the sensors
// (width 8 * rows, height width / 6, Frame360.h:391-392)
static int calib_build_tables(r360_calib* c, int sph_rows = 0, int sph_cols = 0) {
    const int W = sph_cols ? sph_cols : c->rows * 8;
    const int H = sph_rows ? sph_rows : (int)(W * 0.5 * 60.0 / 180);
    c->sph_rows = H; c->sph_cols = W;
    if (c->rows == 0) goto levels;   // sphere-only calibration: no stitch tables
    {
    const float offsetPhi = H / 2 - 0.5;
    const float offsetTheta = -c->rows * 15 / 2 + 0.5;
    const float angle_pixel = 2 * R360_PI / W;
    std::vector<float> sp(H), cp(H), st(W), ct(W);
    for (int r = 0; r < H; ++r) { float phi_i = (offsetPhi - r) * angle_pixel; sp[r] = std::sin(phi_i); cp[r] = std::cos(phi_i); }
    for (int col = 0; col < W; ++col) { float th = (col + offsetTheta) * angle_pixel; st[col] = std::sin(th); ct[col] = std::cos(th); }
    if (upload_floats(&c->d_st_sinphi, sp) || upload_floats(&c->d_st_cosphi, cp) ||
        upload_floats(&c->d_st_sinth, st) || upload_floats(&c->d_st_costh, ct))
        return -1;
    }
levels:
    // pyramid levels of the sphere
    int R = H, C = W, nl = 0;
    for (; nl < R360_MAX_PYR; ++nl) {
        if (R < 2 || C < 8 || (C % 4) != 0) break;
        const float angle_res = 2 * R360_PI / C;
        const float half_nRows = 0.5 * R - 0.5;
        std::vector<float> a(R), b(R), s(C), t(C);
        for (int cc = 0; cc < C; ++cc) { float theta = cc * angle_res; s[cc] = std::sin(theta); t[cc] = std::cos(theta); }
        for (int r = 0; r < R; ++r) { float phi = (half_nRows - r) * angle_res; a[r] = std::sin(phi); b[r] = std::cos(phi); }
        LevelTrig& L = c->trig[nl];
        if (upload_floats(&L.sinphi, a) || upload_floats(&L.cosphi, b) || upload_floats(&L.sinth, s) ||
            upload_floats(&L.costh, t))
            return -1;
        if ((R % 2) || (C % 2)) { ++nl; break; }
        R /= 2; C /= 2;
    }
    c->n_levels = nl;
    return 0;
}

extern "C" int r360_calib_create(r360_ctx* ctx, int rows, int cols, r360_calib** out) {
    CHECK_ARG(ctx && out, "null arg");
    CHECK_ARG(rows > 0 && cols > 0 && rows % 2 == 0 && cols % 2 == 0, "sensor size must be even");
    R360_HIP(hipSetDevice(ctx->device));
    r360_calib* c = new r360_calib;
    c->ctx = ctx; c->rows = rows; c->cols = cols;
    // cameraMatrix: f = 525*cols/640, c = (cols/2-0.5, rows/2-0.5) (CloudRGBD_Ext.h:97-102;
    // equals the QVGA constant of Calib360.h:73-77 and its commented VGA line :83-85)
    const float f = 525 * (float)(cols / 640.0);
    const float cx = cols / 2 - 0.5, cy = rows / 2 - 0.5;
    const float K[9] = {f, 0, 0, 0, f, 0, cx, cy, 1};
    memcpy(c->K, K, sizeof(K));
    for (int k = 0; k < 8; ++k)
        for (int i = 0; i < 16; ++i) c->rt[k][i] = c->rt_inv[k][i] = (i % 5 == 0) ? 1.f : 0.f;
    R360_HIP(hipMalloc(&c->d_rt_inv, sizeof(float) * 128));
    R360_HIP(hipMemcpy(c->d_rt_inv, c->rt_inv, sizeof(float) * 128, hipMemcpyHostToDevice));
    R360_HIP(hipMalloc(&c->d_rt, sizeof(float) * 128));
    R360_HIP(hipMemcpy(c->d_rt, c->rt, sizeof(float) * 128, hipMemcpyHostToDevice));
    if (calib_build_tables(c)) { delete c; return -1; }
    *out = c;
    return 0;
}

// A calibration for spheres given as images (RegisterPhotoICP::setSourceFrame / setTargetFrame(cv::Mat&,
// cv::Mat&), :480-516): no sensors, only the ICP tables of an sph_rows x sph_cols sphere.
extern "C" int r360_calib_create_sphere(r360_ctx* ctx, int sph_rows, int sph_cols, r360_calib** out) {
    CHECK_ARG(ctx && out, "null arg");
    CHECK_ARG(sph_rows >= 2 && sph_cols >= 8 && sph_cols % 8 == 0, "sphere size: rows >= 2, cols a multiple of 8");
    R360_HIP(hipSetDevice(ctx->device));
    r360_calib* c = new r360_calib;
    c->ctx = ctx; c->rows = 0; c->cols = 0;
    for (int k = 0; k < 8; ++k)
        for (int i = 0; i < 16; ++i) c->rt[k][i] = c->rt_inv[k][i] = (i % 5 == 0) ? 1.f : 0.f;
    if (calib_build_tables(c, sph_rows, sph_cols)) { delete c; return -1; }
    *out = c;
    return 0;
}

extern "C" void r360_calib_destroy(r360_calib* c) {
    if (!c) return;
    hipFree(c->d_rt_inv);
    hipFree(c->d_rt);
    hipFree(c->d_st_sinphi); hipFree(c->d_st_cosphi); hipFree(c->d_st_sinth); hipFree(c->d_st_costh);
    for (int l = 0; l < R360_MAX_PYR; ++l) {
        hipFree(c->trig[l].sinphi); hipFree(c->trig[l].cosphi); hipFree(c->trig[l].sinth); hipFree(c->trig[l].costh);
    }
    hipFree(c->clams.d_mult); hipFree(c->clams.d_counts);
    delete c;
}

extern "C" int r360_calib_set_extrinsics(r360_calib* c, const float* rt8) {
    CHECK_ARG(c && rt8, "null arg");
    for (int k = 0; k < 8; ++k) {
        memcpy(c->rt[k], rt8 + 16 * k, sizeof(float) * 16);
        inverse4(c->rt[k], c->rt_inv[k]);                       // Rt_inv = Rt_.inverse() (Calib360.h:129)
    }
    R360_HIP(hipMemcpy(c->d_rt_inv, c->rt_inv, sizeof(float) * 128, hipMemcpyHostToDevice));
    R360_HIP(hipMemcpy(c->d_rt, c->rt, sizeof(float) * 128, hipMemcpyHostToDevice));
    return 0;
}

extern "C" int r360_calib_get_extrinsics(const r360_calib* c, float* rt8, float* rt_inv8, float K[9]) {
    CHECK_ARG(c, "null calib");
    if (rt8) memcpy(rt8, c->rt, sizeof(c->rt));
    if (rt_inv8) memcpy(rt_inv8, c->rt_inv, sizeof(c->rt_inv));
    if (K) memcpy(K, c->K, sizeof(c->K));
    return 0;
}

extern "C" int r360_calib_load_extrinsics(r360_calib* c, const char* dir_in) {
    CHECK_ARG(c, "null arg");
    const std::string dirs = calib_dir_or_default(dir_in, "Extrinsics");
    const char* dir = dirs.c_str();
    float rt[8 * 16];
    for (int k = 0; k < 8; ++k) {
        char path[4096];
        snprintf(path, sizeof(path), "%s/Rt_0%d.txt", dir, k + 1);  // Calib360.h:128
        std::ifstream f(path);
        if (!f) { r360_set_error("cannot open %s", path); return -1; }
        double v[16];
        for (int i = 0; i < 16; ++i)
            if (!(f >> v[i])) { r360_set_error("bad matrix in %s", path); return -1; }
        for (int r = 0; r < 4; ++r)
            for (int cc = 0; cc < 4; ++cc) rt[16 * k + cc * 4 + r] = (float)v[r * 4 + cc];  // text is row-major
    }
    return r360_calib_set_extrinsics(c, rt);
}

// CLAMS model (discrete_depth_distortion_model.cpp:259-280, 82-91) -> per-bin multipliers/counts.
// Accepts the reference's own files (dir/distortion_model{k}) or the compact R360CLAMS1 tables
// (dir/distortion_model{k}.r360, written by tools/compact_clams.py).
static int read_clams(const char* dir, int k, ClamsDev& M, std::vector<float>& mult, std::vector<float>& counts) {
    char path[4096];
    snprintf(path, sizeof(path), "%s/distortion_model%d", dir, k + 1);
    std::ifstream in(path, std::ios::binary);
    bool compact = false;
    if (!in) {
        snprintf(path, sizeof(path), "%s/distortion_model%d.r360", dir, k + 1);
        in.open(path, std::ios::binary);
        compact = true;
    }
    if (!in) { r360_set_error("cannot open %s/distortion_model%d[.r360]", dir, k + 1); return -1; }
    std::string line;
    std::getline(in, line);
    int w, h, bw, bh, nx, ny, nb = 0; double bd;
    if (compact) {
        if (line != "R360CLAMS1") { r360_set_error("bad compact CLAMS header in %s", path); return -1; }
        in.read((char*)&w, 4); in.read((char*)&h, 4); in.read((char*)&bw, 4); in.read((char*)&bh, 4);
        in.read((char*)&nx, 4); in.read((char*)&ny, 4); in.read((char*)&nb, 4); in.read((char*)&bd, 8);
        std::vector<float> c((size_t)nx * ny * nb), m((size_t)nx * ny * nb);
        in.read((char*)c.data(), 4 * c.size());
        in.read((char*)m.data(), 4 * m.size());
        if (!in) { r360_set_error("truncated %s", path); return -1; }
        counts.insert(counts.end(), c.begin(), c.end());
        mult.insert(mult.end(), m.begin(), m.end());
    } else {
        if (line != "DiscreteDepthDistortionModel v01") { r360_set_error("bad CLAMS header in %s", path); return -1; }
        in.read((char*)&w, 4); in.read((char*)&h, 4); in.read((char*)&bw, 4); in.read((char*)&bh, 4);
        in.read((char*)&bd, 8); in.read((char*)&nx, 4); in.read((char*)&ny, 4);
        if (!in) { r360_set_error("truncated %s", path); return -1; }
        for (int i = 0; i < nx * ny; ++i) {
            double maxd, bdep;
            in.read((char*)&maxd, 8); in.read((char*)&nb, 4); in.read((char*)&bdep, 8);
            std::vector<float> vec[4];
            for (int q = 0; q < 4; ++q) {
                int bytes, rr, cc;
                in.read((char*)&bytes, 4); in.read((char*)&rr, 4); in.read((char*)&cc, 4);
                vec[q].resize((size_t)rr * cc);
                in.read((char*)vec[q].data(), 4 * vec[q].size());
            }
            if (!in || vec[0].size() != (size_t)nb || vec[3].size() != (size_t)nb) {
                r360_set_error("bad frustum in %s", path); return -1;
            }
            for (int b = 0; b < nb; ++b) { counts.push_back(vec[0][b]); mult.push_back(vec[3][b]); }
        }
    }
    // downsampleParams(2) (Calib360.h:115, discrete_depth_distortion_model.cpp:313-320)
    M.width = w / 2; M.height = h / 2; M.bin_w = bw / 2; M.bin_h = bh / 2; M.nx = nx; M.ny = ny;
    M.num_bins = nb; M.bin_depth = bd;
    return 0;
}

extern "C" int r360_calib_load_intrinsics(r360_calib* c, const char* dir_in) {
    CHECK_ARG(c, "null arg");
    const std::string dirs = calib_dir_or_default(dir_in, "Intrinsics");
    const char* dir = dirs.c_str();
    std::vector<float> mult, counts;
    for (int k = 0; k < 8; ++k)
        if (read_clams(dir, k, c->clams, mult, counts)) return -1;
    if (upload_floats(&c->clams.d_mult, mult) || upload_floats(&c->clams.d_counts, counts)) return -1;
    c->has_intrinsics = true;
    return 0;
}

// ------------------------------------------------------------------ Frame360
extern "C" int r360_frame_create(r360_ctx* ctx, const r360_calib* calib, r360_frame** out) {
    CHECK_ARG(ctx && calib && out, "null arg");
    R360_HIP(hipSetDevice(ctx->device));
    r360_frame* f = new r360_frame;
    f->ctx = ctx; f->calib = calib;
    f->rows = calib->rows; f->cols = calib->cols;
    f->sph_rows = calib->sph_rows; f->sph_cols = calib->sph_cols;
    f->n_levels = calib->n_levels;
    const size_t ns = (size_t)8 * f->rows * f->cols, nsph = (size_t)f->sph_rows * f->sph_cols;
    if (ns) {                        // a sphere-only frame (r360_calib_create_sphere) has no sensor images
        R360_HIP(hipMalloc(&f->d_bgr, ns * 3));
        R360_HIP(hipMalloc(&f->d_depth, ns * 2));
        R360_HIP(hipMalloc(&f->d_depth_m, ns * 4));
    }
    R360_HIP(hipMalloc(&f->d_sph_bgr, nsph * 3));
    R360_HIP(hipMalloc(&f->d_sph_depth, nsph * 2));
    int R = f->sph_rows, C = f->sph_cols;
    for (int l = 0; l < f->n_levels; ++l) {
        f->lv[l].rows = R; f->lv[l].cols = C;
        R360_HIP(hipMalloc(&f->lv[l].p0, sizeof(float2) * (size_t)R * C));
        R360_HIP(hipMalloc(&f->lv[l].tg, sizeof(float4) * (size_t)R * C));
        R360_HIP(hipMalloc(&f->lv[l].pts, sizeof(float4) * (size_t)R * C));
        if (l == 0) R360_HIP(hipMalloc(&f->lv[l].pk, sizeof(uint32_t) * (size_t)R * C));
        R /= 2; C /= 2;
    }
    f->src_blocks = (int)((nsph + R360_SRC_BLOCK - 1) / R360_SRC_BLOCK);
    R360_HIP(hipMalloc(&f->d_npts, sizeof(int) * R360_MAX_PYR));
    R360_HIP(hipMemsetAsync(f->d_npts, 0, sizeof(int) * R360_MAX_PYR, f->ctx->stream));
    R360_HIP(hipMalloc(&f->d_src_cnt, sizeof(int) * R360_MAX_PYR * (size_t)f->src_blocks));
    SrcLevel sl[R360_MAX_PYR];
    for (int l = 0; l < f->n_levels; ++l) {
        const LevelTrig& T = calib->trig[l];
        sl[l] = SrcLevel{f->lv[l].p0, f->lv[l].pts, T.sinphi, T.cosphi, T.sinth, T.costh, f->lv[l].rows, f->lv[l].cols};
    }
    R360_HIP(hipMalloc(&f->d_src_levels, sizeof(SrcLevel) * R360_MAX_PYR));
    R360_HIP(hipMemcpy(f->d_src_levels, sl, sizeof(SrcLevel) * f->n_levels, hipMemcpyHostToDevice));
    R360_HIP(hipEventCreateWithFlags(&f->bgr_ev, hipEventDisableTiming));
    *out = f;
    return 0;
}

// The event recorded on a frame's stream right after its last pyramid build (r360_frame_build_async).  The dense
// queue's batches wait on it instead of on the stream's tail at submit time, which by then also held the next
// frame's upload (a pipeline prefetches it right after the build).  Kept beside the frame (keyed by its address).
static std::mutex g_bev_m;
static std::unordered_map<const r360_frame*, hipEvent_t> g_bev;

hipEvent_t frame_build_event(const r360_frame* f) {
    std::lock_guard<std::mutex> lk(g_bev_m);
    auto it = g_bev.find(f);
    return it == g_bev.end() ? nullptr : it->second;
}

static int frame_build_event_record(const r360_frame* f) {
    hipEvent_t e = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_bev_m);
        auto it = g_bev.find(f);
        if (it != g_bev.end()) e = it->second;
    }
    if (!e) {
        R360_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        std::lock_guard<std::mutex> lk(g_bev_m);
        g_bev[f] = e;
    }
    R360_HIP(hipEventRecord(e, f->ctx->stream));
    const_cast<r360_frame*>(f)->build_gen.fetch_add(1, std::memory_order_release);
    return 0;
}

extern "C" void r360_frame_destroy(r360_frame* f) {
    if (!f) return;
    {
        std::lock_guard<std::mutex> lk(g_bev_m);
        auto it = g_bev.find(f);
        if (it != g_bev.end()) {
            (void)hipEventDestroy(it->second);
            g_bev.erase(it);
        }
    }
    // hipFree synchronises the device; the frame never dereferences its ctx here so frames may
    // outlive their context at interpreter shutdown.
    hipFree(f->d_bgr); hipFree(f->d_depth); hipFree(f->d_depth_m); hipFree(f->d_sph_bgr); hipFree(f->d_sph_depth);
    for (int l = 0; l < R360_MAX_PYR; ++l) { hipFree(f->lv[l].p0); hipFree(f->lv[l].tg); hipFree(f->lv[l].pts); hipFree(f->lv[l].pk); }
    hipFree(f->d_npts); hipFree(f->d_src_cnt); hipFree(f->d_src_levels);
    for (int l = 0; l < f->n_slevels; ++l) { hipFree(f->sp[l].p0); hipFree(f->sp[l].tg); }
    plane_bufs_free(f);
    if (f->bgr_ev) hipEventDestroy(f->bgr_ev);
    delete f->sphere_cloud;
    delete f;
}

// The sensor images into the frame.  With ctx->split_upload the depth goes first, on the ctx stream, and the BGR images
// follow on the ctx's upload stream, after the depth copy and after everything the ctx stream had enqueued before (the
// previous build's readers of d_bgr), so the undistortion and the plane stage's geometric part start one copy earlier
// (the colours are first read by launch_rgb, behind f->bgr_ev).  Otherwise both on the ctx stream, and nothing waits
// on an event (throughput runs: the waits measured 6 % of the headline, profiles/r6_split).
static int frame_copy_images(r360_frame* f, const void* bgr8, const void* depth8, hipMemcpyKind kind) {
    r360_ctx* ctx = f->ctx;
    const size_t ns = (size_t)8 * f->rows * f->cols;
    if (ctx->split_upload) {
        R360_HIP(hipMemcpyAsync(f->d_depth, depth8, ns * 2, kind, ctx->stream));
        if (!ctx->up_stream) {
            R360_HIP(hipStreamCreateWithFlags(&ctx->up_stream, hipStreamNonBlocking));
            R360_HIP(hipEventCreateWithFlags(&ctx->up_ev, hipEventDisableTiming));
        }
        R360_HIP(hipEventRecord(ctx->up_ev, ctx->stream));
        R360_HIP(hipStreamWaitEvent(ctx->up_stream, ctx->up_ev, 0));
        R360_HIP(hipMemcpyAsync(f->d_bgr, bgr8, ns * 3, kind, ctx->up_stream));
        R360_HIP(hipEventRecord(f->bgr_ev, ctx->up_stream));
        f->bgr_split = true;
    } else {
        if (hipEvent_t e = f->bgr_wait()) R360_HIP(hipStreamWaitEvent(ctx->stream, e, 0));   // an earlier split copy
        R360_HIP(hipMemcpyAsync(f->d_bgr, bgr8, ns * 3, kind, ctx->stream));
        R360_HIP(hipMemcpyAsync(f->d_depth, depth8, ns * 2, kind, ctx->stream));
        f->bgr_split = false;
    }
    return 0;
}

extern "C" int r360_frame_upload(r360_frame* f, const uint8_t* bgr8, const uint16_t* depth8) {
    CHECK_ARG(f && bgr8 && depth8, "null arg");
    if (f && bind_device(f->ctx->device)) return -1;
    CHECK_ARG(f->rows > 0, "a sphere-only frame has no sensor images");
    planes_join(f);   // a plane stage still reading the images (a plane queue's batch) ends first
    if (frame_copy_images(f, bgr8, depth8, hipMemcpyHostToDevice)) return -1;
    R360_HIP(hipStreamSynchronize(f->ctx->stream));
    if (hipEvent_t e = f->bgr_wait()) R360_HIP(hipEventSynchronize(e));
    f->built = 0;
    return 0;
}

// Enqueued on the ctx stream (and its upload stream); the host buffers must stay valid until the streams reach the
// copies (page-locked buffers, r360_host_register, make the copies truly asynchronous).
extern "C" int r360_frame_upload_async(r360_frame* f, const uint8_t* bgr8, const uint16_t* depth8) {
    CHECK_ARG(f && bgr8 && depth8, "null arg");
    if (f && bind_device(f->ctx->device)) return -1;
    CHECK_ARG(f->rows > 0, "a sphere-only frame has no sensor images");
    planes_join(f);   // a plane stage still reading the images (a plane queue's batch) ends first
    if (frame_copy_images(f, bgr8, depth8, hipMemcpyHostToDevice)) return -1;
    f->built = 0;
    return 0;
}

extern "C" int r360_host_register(void* p, size_t bytes) {
    CHECK_ARG(p && bytes, "null arg");
    R360_HIP(hipHostRegister(p, bytes, hipHostRegisterDefault));
    return 0;
}

extern "C" int r360_host_unregister(void* p) {
    CHECK_ARG(p, "null arg");
    R360_HIP(hipHostUnregister(p));
    return 0;
}

// setSourceFrame / setTargetFrame(cv::Mat& imgRGB, cv::Mat& imgDepth) (RegisterPhotoICP.h:480-516): a sphere
// given as images (BGR u8 sph_rows x sph_cols x 3, range u16 mm) replaces the frame's sphere; its pyramid
// (gray, depth, gradients with the seam mask, source points) is rebuilt.
extern "C" int r360_frame_set_sphere(r360_frame* f, const uint8_t* bgr, const uint16_t* range_mm, int sph_rows,
                                     int sph_cols) {
    CHECK_ARG(f && bgr && range_mm, "null arg");
    if (f && bind_device(f->ctx->device)) return -1;
    CHECK_ARG(sph_rows == f->sph_rows && sph_cols == f->sph_cols,
              "sphere size differs from the frame's (create it from r360_calib_create_sphere)");
    const size_t n = (size_t)sph_rows * sph_cols;
    R360_HIP(hipMemcpyAsync(f->d_sph_bgr, bgr, n * 3, hipMemcpyHostToDevice, f->ctx->stream));
    R360_HIP(hipMemcpyAsync(f->d_sph_depth, range_mm, n * 2, hipMemcpyHostToDevice, f->ctx->stream));
    if (launch_sphere_level0(f) || launch_pyramid(f) || frame_build_event_record(f)) return -1;
    R360_HIP(hipStreamSynchronize(f->ctx->stream));
    f->built = (f->built & ~(unsigned)(R360_BUILD_SPHERE | R360_BUILD_PYRAMID)) | R360_BUILD_SPHERE | R360_BUILD_PYRAMID;
    return 0;
}

extern "C" int r360_frame_upload_device(r360_frame* f, const void* d_bgr8, const void* d_depth8) {
    CHECK_ARG(f && d_bgr8 && d_depth8, "null arg");
    if (f && bind_device(f->ctx->device)) return -1;
    CHECK_ARG(f->rows > 0, "a sphere-only frame has no sensor images");
    planes_join(f);   // a plane stage still reading the images (a plane queue's batch) ends first
    const size_t ns = (size_t)8 * f->rows * f->cols;
    if (hipEvent_t e = f->bgr_wait()) R360_HIP(hipStreamWaitEvent(f->ctx->stream, e, 0));   // an earlier split copy
    R360_HIP(hipMemcpyAsync(f->d_bgr, d_bgr8, ns * 3, hipMemcpyDeviceToDevice, f->ctx->stream));
    f->bgr_split = false;
    R360_HIP(hipMemcpyAsync(f->d_depth, d_depth8, ns * 2, hipMemcpyDeviceToDevice, f->ctx->stream));
    f->built = 0;
    return 0;
}

extern "C" int r360_frame_build_async(r360_frame* f, unsigned flags) {
    CHECK_ARG(f, "null frame");
    if (f && bind_device(f->ctx->device)) return -1;
    CHECK_ARG(f->rows > 0 || flags == 0, "a sphere-only frame has no sensor images to build from (r360_frame_set_sphere)");
    if (flags & (R360_BUILD_UNDISTORT | R360_BUILD_CLOUD | R360_BUILD_PLANES)) {
        // the previous build's plane stage may run on another stream (plane queue, r360_frames_build) and read the
        // undistorted depth: its assembly thread has waited for it
        planes_join(f);
        if (launch_undistort(f)) return -1;
        f->built |= R360_BUILD_UNDISTORT;
    }
    // the plane stage first: its results go to the host (PbMap assembly, then RegisterPbMap), which the dense
    // stage waits for anyway, so the stitch and pyramid run on the GPU while the host assembles and matches
    if (flags & (R360_BUILD_CLOUD | R360_BUILD_PLANES)) {
        // buildSphereCloud + getPlanes (Frame360.h:467-510, 615-640): the per-pixel part is enqueued
        // here; the per-plane PbMap assembly runs on the host when the planes are first needed
        if (planes_enqueue(f)) return -1;
        f->built |= R360_BUILD_CLOUD | R360_BUILD_PLANES;
        delete f->sphere_cloud;  // a cloud set by loadCloud is replaced by the built one
        f->sphere_cloud = nullptr;
    }
    if (flags & (R360_BUILD_SPHERE | R360_BUILD_PYRAMID)) {
        if (launch_stitch(f)) return -1;
        f->built |= R360_BUILD_SPHERE;
    }
    if (flags & R360_BUILD_PYRAMID) {
        if (launch_pyramid(f)) return -1;
        f->built |= R360_BUILD_PYRAMID;
        if (frame_build_event_record(f)) return -1;
    }
    if (flags & R360_BUILD_SENSOR_PYRAMID) {
        if (launch_sensor_pyramid(f)) return -1;
        f->built |= R360_BUILD_SENSOR_PYRAMID;
    }
    return 0;
}

extern "C" int r360_frame_build(r360_frame* f, unsigned flags) {
    int rc = r360_frame_build_async(f, flags);
    if (rc) return rc;
    if (flags & R360_BUILD_PLANES) return planes_finish(f);
    R360_HIP(hipStreamSynchronize(f->ctx->stream));
    return 0;
}

// RegisterPhotoICP::setNumPyr (RegisterPhotoICP.h:224-227) fixes how many pyramid levels setSourceFrame /
// setTargetFrame build: a frame builds the calibration's full depth unless told to stop at n levels (its buffers for
// the deeper levels stay allocated, unused).  Clears the frame's built stages.
extern "C" int r360_frame_set_levels(r360_frame* f, int n) {
    CHECK_ARG(f && f->calib, "null frame");
    CHECK_ARG(n >= 1 && n <= f->calib->n_levels, "levels must be 1 .. the calibration's pyramid depth");
    planes_join(f);
    f->n_levels = n;
    f->built = 0;
    return 0;
}

extern "C" int r360_frame_set_compaction(r360_frame* f, int all) {
    CHECK_ARG(f, "null frame");
    f->compact_all = all != 0;
    return 0;
}

extern "C" int r360_frame_dims(const r360_frame* f, int* rows, int* cols, int* sph_rows, int* sph_cols) {
    CHECK_ARG(f, "null frame");
    if (rows) *rows = f->rows;
    if (cols) *cols = f->cols;
    if (sph_rows) *sph_rows = f->sph_rows;
    if (sph_cols) *sph_cols = f->sph_cols;
    return 0;
}

extern "C" int r360_frame_built(const r360_frame* f, unsigned* flags) {
    CHECK_ARG(f && flags, "null arg");
    *flags = f->built.load();
    return 0;
}

extern "C" int r360_frame_get_sphere(r360_frame* f, uint8_t* bgr, uint16_t* depth) {
    CHECK_ARG(f, "null frame");
    CHECK_ARG(f->built & R360_BUILD_SPHERE, "sphere not built");
    const size_t n = (size_t)f->sph_rows * f->sph_cols;
    R360_HIP(hipStreamSynchronize(f->ctx->stream));
    if (bgr) R360_HIP(hipMemcpy(bgr, f->d_sph_bgr, n * 3, hipMemcpyDeviceToHost));
    if (depth) R360_HIP(hipMemcpy(depth, f->d_sph_depth, n * 2, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int r360_frame_get_depth_m(r360_frame* f, float* depth8) {
    CHECK_ARG(f && depth8, "null arg");
    CHECK_ARG(f->built & R360_BUILD_UNDISTORT, "undistorted depth not built");
    R360_HIP(hipStreamSynchronize(f->ctx->stream));
    R360_HIP(hipMemcpy(depth8, f->d_depth_m, sizeof(float) * 8 * f->rows * f->cols, hipMemcpyDeviceToHost));
    return 0;
}

static int copy_level(r360_frame* f, const float2* d_p0, const float4* d_tg, int R, int C, int* rows, int* cols,
                      float* gray, float* depth, float* gx, float* gy, float* dgx, float* dgy) {
    if (rows) *rows = R;
    if (cols) *cols = C;
    const size_t n = (size_t)R * C;
    R360_HIP(hipStreamSynchronize(f->ctx->stream));
    std::vector<float2> p0(n);
    std::vector<float4> tg(n);
    R360_HIP(hipMemcpy(p0.data(), d_p0, n * sizeof(float2), hipMemcpyDeviceToHost));
    R360_HIP(hipMemcpy(tg.data(), d_tg, n * sizeof(float4), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; ++i) {
        if (gray) gray[i] = p0[i].x;
        if (depth) depth[i] = p0[i].y;
        if (gx) gx[i] = tg[i].x;
        if (gy) gy[i] = tg[i].y;
        if (dgx) dgx[i] = tg[i].z;
        if (dgy) dgy[i] = tg[i].w;
    }
    return 0;
}

extern "C" int r360_frame_get_level(r360_frame* f, int level, int* rows, int* cols, float* gray, float* depth,
                                    float* gx, float* gy, float* dgx, float* dgy) {
    CHECK_ARG(f, "null frame");
    CHECK_ARG(level >= 0 && level < f->n_levels, "level out of range");
    CHECK_ARG(f->built & R360_BUILD_PYRAMID, "pyramid not built");
    const LevelBufs& L = f->lv[level];
    return copy_level(f, L.p0, L.tg, L.rows, L.cols, rows, cols, gray, depth, gx, gy, dgx, dgy);
}

extern "C" int r360_frame_get_points(r360_frame* f, int level, float* xyzg, int cap, int* n) {
    CHECK_ARG(f && n, "null arg");
    CHECK_ARG(level >= 0 && level < f->n_levels, "level out of range");
    CHECK_ARG(f->built & R360_BUILD_PYRAMID, "pyramid not built");
    if (!((f->compacted >> level) & 1u)) {   // a level batched passes stream as an image: compacted on request
        if (int rc = launch_src_compaction(f, 1u << level)) return rc;
        f->compacted |= 1u << level;
    }
    int np = 0;
    R360_HIP(hipMemcpyAsync(&np, f->d_npts + level, sizeof(int), hipMemcpyDeviceToHost, f->ctx->stream));
    R360_HIP(hipStreamSynchronize(f->ctx->stream));
    *n = np;
    if (xyzg && cap > 0) {
        const int m = np < cap ? np : cap;
        R360_HIP(hipMemcpy(xyzg, f->lv[level].pts, sizeof(float4) * (size_t)m, hipMemcpyDeviceToHost));
    }
    return 0;
}

extern "C" int r360_frame_get_sensor_level(r360_frame* f, int sensor, int level, int* rows, int* cols, float* gray,
                                           float* depth, float* gx, float* gy, float* dgx, float* dgy) {
    CHECK_ARG(f, "null frame");
    CHECK_ARG(f->built & R360_BUILD_SENSOR_PYRAMID, "sensor pyramid not built (R360_BUILD_SENSOR_PYRAMID)");
    CHECK_ARG(level >= 0 && level < f->n_slevels, "level out of range");
    CHECK_ARG(sensor >= 0 && sensor < 8, "sensor out of range");
    const LevelBufs& L = f->sp[level];
    const size_t off = (size_t)sensor * L.rows * L.cols;
    return copy_level(f, L.p0 + off, L.tg + off, L.rows, L.cols, rows, cols, gray, depth, gx, gy, dgx, dgy);
}

// ------------------------------------------------------------------ RegisterPhotoICP
extern "C" void r360_icp_default_params(r360_icp_params* p) {
    p->n_pyr = 4;                  // RegisterPhotoICP() (:204)
    p->max_iters = 10;             // :4593
    p->min_depth = 0.3f;
    p->max_depth = 6.0f;
    p->std_dev_photo = (float)(6. / 255);
    p->std_dev_depth = 0.2f;
    p->thres_sal_int = 0.01f;
    p->thres_sal_depth = 0.01f;
    p->tol_residual = 1e-3;
    p->tol_update = 1e-4;
    p->lambda = 1.0;
    p->fixed_iters_level0 = 0;
}

static IcpConst make_const(const r360_icp_params* p, int level, int n_pixels, int occ = 0) {
    IcpConst C;
    memset(&C, 0, sizeof(C));
    C.min_d = p->min_depth; C.max_d = p->max_depth;
    C.sd_photo = p->std_dev_photo; C.sd_depth = p->std_dev_depth;
    C.thr_int = p->thres_sal_int; C.thr_depth = p->thres_sal_depth;
    C.sd_photo_inv_f = (float)(1. / p->std_dev_photo);
    C.sd_photo_inv_d = 1. / p->std_dev_photo;
    C.tol_res = p->tol_residual; C.tol_upd = p->tol_update; C.lambda = p->lambda;
    C.max_iters = p->max_iters; C.fixed_iters0 = p->fixed_iters_level0;
    // diagnostic only (tools/stamps.py ALIGN=1): the device GN expects more level-0 iterations than are launched,
    // so the last launched pass is a continuing one
    static const int diag_extra = R360_KNOB("R360_DIAG_EXTRA_ITERS", 0);
    if (C.fixed_iters0 > 0) C.fixed_iters0 += diag_extra;
    C.n_pixels = n_pixels; C.level = level; C.occ = occ;
    return C;
}

static int check_pair(r360_ctx* ctx, r360_frame* trg, r360_frame* src, const r360_icp_params* p) {
    CHECK_ARG(ctx && trg && src && p, "null arg");
    CHECK_ARG(trg->sph_rows == src->sph_rows && trg->sph_cols == src->sph_cols, "frame size mismatch");
    CHECK_ARG((trg->built & R360_BUILD_PYRAMID) && (src->built & R360_BUILD_PYRAMID),
              "frames need R360_BUILD_PYRAMID (setSourceFrame/setTargetFrame)");
    CHECK_ARG(p->n_pyr >= 1 && p->n_pyr <= src->n_levels, "n_pyr exceeds the frame's pyramid depth");
    CHECK_ARG(p->min_depth == 0.3f && p->max_depth == 6.0f,
              "non-default min/max depth changes the depth pyramid: not supported in this version");
    CHECK_ARG(ctx->partials_cap >= icp_blocks_for(src->lv[0].rows * src->lv[0].cols), "partials buffer too small");
    return 0;
}

// Replays the captured pass sequence of (trg, src, method, p) on ctx's stream, capturing it on first use.  The key
// holds everything the launches read besides device memory contents: the frames' level buffers and sizes, the
// sphere tables, the ctx's state / record / counter / queue buffers, the method and the parameters.
template <class Enqueue>
static int align_graph_launch(r360_ctx* ctx, const r360_frame* trg, const r360_frame* src, int method,
                              const r360_icp_params* p, bool persist, Enqueue&& enqueue) {
    std::vector<uintptr_t> key;
    key.reserve(16 + 20 * p->n_pyr);
    auto put = [&](const void* q) { key.push_back((uintptr_t)q); };
    put(trg); put(src); key.push_back((uintptr_t)method); key.push_back((uintptr_t)persist);
    put(ctx->d_state); put(ctx->d_partials); put(ctx->d_gticket); put(ctx->d_defer);
    key.push_back((uintptr_t)ctx->defer_cap); key.push_back((uintptr_t)ctx->partials_cap); put(ctx->d_ktime);
    put(src->d_npts); put(src->calib);
    {
        uintptr_t w[(sizeof(r360_icp_params) + sizeof(uintptr_t) - 1) / sizeof(uintptr_t)] = {};
        memcpy(w, p, sizeof(r360_icp_params));
        for (uintptr_t x : w) key.push_back(x);
    }
    for (int l = 0; l < p->n_pyr; ++l) {
        for (const r360_frame* f : {trg, src}) {
            const LevelBufs& L = f->lv[l];
            key.push_back(((uintptr_t)(unsigned)L.rows << 32) | (unsigned)L.cols);
            put(L.p0); put(L.tg); put(L.pts); put(L.pk);
        }
        const LevelTrig& T = src->calib->trig[l];
        put(T.sinphi); put(T.cosphi); put(T.sinth); put(T.costh);
    }
    ++ctx->graph_clock;
    for (auto& g : ctx->graphs)
        if (g.key == key) {
            g.used = ctx->graph_clock;
            R360_HIP(hipGraphLaunch(g.exec, ctx->stream));
            return 0;
        }
    hipGraph_t graph = nullptr;
    // captured on the ctx's capture stream (the launchers enqueue on ctx->stream, pointed at it meanwhile)
    hipStream_t cs = capture_stream(ctx);
    if (!cs) return -1;
    hipStream_t own = ctx->stream;
    R360_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed));
    ctx->stream = cs;
    const int rc = enqueue();
    ctx->stream = own;
    const hipError_t ec = hipStreamEndCapture(cs, &graph);
    if (rc) { if (graph) (void)hipGraphDestroy(graph); return rc; }
    R360_HIP(ec);
    hipGraphExec_t exec = nullptr;
    const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    R360_HIP(ei);
    constexpr size_t kMaxGraphs = 8;   // e.g. the ordered pairs of three rotating frame buffers
    if (ctx->graphs.size() >= kMaxGraphs) {
        size_t lru = 0;
        for (size_t i = 1; i < ctx->graphs.size(); ++i)
            if (ctx->graphs[i].used < ctx->graphs[lru].used) lru = i;
        R360_HIP(hipStreamSynchronize(ctx->stream));   // the evicted graph may still be running
        (void)hipGraphExecDestroy(ctx->graphs[lru].exec);
        ctx->graphs.erase(ctx->graphs.begin() + (long)lru);
    }
    ctx->graphs.push_back({std::move(key), exec, ctx->graph_clock});
    R360_HIP(hipGraphLaunch(exec, ctx->stream));
    return 0;
}

// One persistent level launch in flight per process: its grid must be resident whole (k_icp_level), and two of
// them leave room per CU (icp_level_persist_ok keeps one workgroup per CU spare); the slot is taken when an
// alignment is enqueued that way and given back when its result is read (or the ctx is destroyed).  Another
// alignment enqueued meanwhile launches its passes one by one.
static std::atomic<int> g_persist_slot{0};
static bool persist_take(r360_ctx* ctx) {
    if (ctx->persist_held) return true;
    int z = 0;
    if (!g_persist_slot.compare_exchange_strong(z, 1)) return false;
    ctx->persist_held = 1;
    return true;
}
void persist_release(r360_ctx* ctx) {
    if (!ctx->persist_held) return;
    ctx->persist_held = 0;
    g_persist_slot.store(0);
}

extern "C" int r360_align360_async(r360_ctx* ctx, r360_frame* trg, r360_frame* src, const float init[16], int method,
                                   int occlusion, const r360_icp_params* p) {
    if (ctx && bind_device(ctx->device)) return -1;
    if (int rc = check_pair(ctx, trg, src, p)) return rc;
    CHECK_ARG(init, "null init pose");
    CHECK_ARG(method >= 0 && method <= 2, "invalid method");
    CHECK_ARG(occlusion >= 0 && occlusion <= 2, "occlusion must be 0, 1 or 2");
    if (ensure_defer(ctx, src->lv[0].rows * src->lv[0].cols)) return -1;
    // frames built on another context (another thread's): this stream waits for their pyramid builds
    for (const r360_frame* f : {trg, src})
        if (f->ctx != ctx)
            if (hipEvent_t e = frame_build_event(f)) R360_HIP(hipStreamWaitEvent(ctx->stream, e, 0));
    IcpState* h = ctx->h_state;
    ctx->align_t0 = now_s();
    memset(h, 0, sizeof(IcpState));
    memcpy(h->pose, init, sizeof(float) * 16);
    memcpy(h->cand, init, sizeof(float) * 16);
    h->dbg[8] = ~0ull;
    R360_HIP(hipMemcpyAsync(ctx->d_state, h, sizeof(IcpState), hipMemcpyHostToDevice, ctx->stream));
    // with r360_ctx_persistent_levels(ctx, 1) the plain pass without per-launch timing events runs each level as
    // one persistent launch (k_icp_level) when every level's grid fits; otherwise (the default, occlusion variants,
    // timing, another persistent launch in flight) one launch per pass.  R360_PERSIST=1 (experiment builds) sets
    // the option for every context.
    static const bool persist_env = R360_KNOB("R360_PERSIST", 0) != 0;
    // R360_PERSIST_MIN_LEVEL (experiment builds): only levels >= it run persistent, the finer ones pass by pass
    static const int persist_min = R360_KNOB("R360_PERSIST_MIN_LEVEL", 0);
    bool persist = (ctx->persist_levels || persist_env) && !occlusion && !ctx->timing && !R360_POLL;
    for (int l = persist_min; persist && l < p->n_pyr; ++l) persist = icp_level_persist_ok(ctx, src, l, method);
    if (persist) persist = persist_take(ctx);
    auto passes_of = [&]() -> int {
        for (int l = p->n_pyr - 1; l >= 0; --l) {
            const int np = src->lv[l].rows * src->lv[l].cols;
            const IcpConst C = make_const(p, l, np, occlusion);
            const int passes = 1 + ((l == 0 && p->fixed_iters_level0 > 0) ? p->fixed_iters_level0 : p->max_iters);
            if (persist && l >= persist_min) {
                if (launch_icp_level_persist(ctx, trg, src, l, method, C, passes)) return -1;
                continue;
            }
            for (int k = 0; k < passes; ++k)
                if (launch_icp_level(ctx, trg, src, l, method, C, k == 0, 0)) return -1;
        }
        return 0;
    };
    // graphs for the plain pass (occlusion passes size their buffers on first use) without per-launch timing
    // events; R360_NO_GRAPH=1 launches one by one (A/B)
    static const bool no_graph = R360_KNOB("R360_NO_GRAPH", 0) != 0;
    int rc;
    if (no_graph || R360_POLL || occlusion || ctx->timing) rc = passes_of();
    else rc = align_graph_launch(ctx, trg, src, method, p, persist, passes_of);
    if (rc) {
        persist_release(ctx);
        return -1;
    }
    ctx->async_nL = p->n_pyr;
    ctx->async_persist = persist ? 1 : 0;
    ctx->async_pending = 1;
    return 0;
}

static void fill_stats(const IcpState* h, r360_icp_stats* st) {
    memset(st, 0, sizeof(*st));
    for (int l = 0; l < 8; ++l) { st->iters[l] = h->iters[l]; st->evals[l] = h->evals_l[l]; }
    st->illposed = h->illposed;
    st->sso = h->sso;
    st->error = h->error;
    st->passes = h->passes;
    st->av_photo_residual = h->av_photo;
    st->av_depth_residual = h->av_depth;
    st->av_residual = h->av_res;
    st->residuals_set = h->av_set & 3;
}

extern "C" int r360_align360_result(r360_ctx* ctx, float pose_out[16], float H_out[36], float g_out[6],
                                    r360_icp_stats* st) {
    CHECK_ARG(ctx && ctx->async_pending, "no alignment pending");
    IcpState* h = ctx->h_state;
    R360_HIP(hipMemcpyAsync(h, ctx->d_state, sizeof(IcpState), hipMemcpyDeviceToHost, ctx->stream));
    bool waited = false;
    const int wrc = align_wait(ctx, &waited);
    if (wrc == 0 && waited) ctx->align_est = now_s() - ctx->align_t0;   // the next alignment's wait plan
    persist_release(ctx);
    if (wrc) return -1;
    ctx->async_pending = 0;
    if (h->fault) {
        // the drained grid left the group arrival counters part-way (only a pass's step workgroup resets them): zero
        // them so the next alignment on this ctx picks the right last workgroup (the pass ticket lives in the state,
        // which every alignment re-uploads)
        R360_HIP(hipMemsetAsync(ctx->d_gticket, 0, sizeof(unsigned) * R360_TICKET_STRIDE * R360_TICKET_GROUPS,
                                ctx->stream));
        R360_HIP(hipStreamSynchronize(ctx->stream));
        r360_set_error("alignFrames360: a persistent level launch timed out waiting for a pass (GPU oversubscribed?)");
        return -1;
    }
    if (pose_out) memcpy(pose_out, h->pose, sizeof(float) * 16);
    if (H_out) memcpy(H_out, h->Hout, sizeof(float) * 36);
    if (g_out) memcpy(g_out, h->gout, sizeof(float) * 6);
    if (st) {
        fill_stats(h, st);
        st->persistent = ctx->async_persist;
    }
    return h->illposed ? 1 : 0;
}

extern "C" int r360_align360(r360_ctx* ctx, r360_frame* trg, r360_frame* src, const float init[16], int method,
                             int occlusion, const r360_icp_params* p, float pose_out[16], float H_out[36],
                             float g_out[6], r360_icp_stats* st) {
    if (int rc = r360_align360_async(ctx, trg, src, init, method, occlusion, p)) return rc;
    return r360_align360_result(ctx, pose_out, H_out, g_out, st);
}

int align360_batch_enqueue(r360_ctx* ctx, int n, r360_frame* const* trg, r360_frame* const* src, const float* init,
                           int method, const r360_icp_params* p, bool wait_frames);

// Makes ctx's stream wait for the work already enqueued on the streams of the frames' contexts (their builds)
int ctx_wait_frames(r360_ctx* ctx, r360_frame* const* frames, int n) {
    std::vector<hipStream_t> seen;
    for (int i = 0; i < n; ++i) {
        hipStream_t s = frames[i]->ctx->stream;
        if (s == ctx->stream) continue;
        bool dup = false;
        for (hipStream_t t : seen) dup = dup || t == s;
        if (dup) continue;
        seen.push_back(s);
    }
    while (ctx->sync_ev.size() < seen.size()) {
        hipEvent_t e;
        R360_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->sync_ev.push_back(e);
    }
    for (size_t i = 0; i < seen.size(); ++i) {
        R360_HIP(hipEventRecord(ctx->sync_ev[i], seen[i]));
        R360_HIP(hipStreamWaitEvent(ctx->stream, ctx->sync_ev[i], 0));
    }
    return 0;
}

extern "C" int r360_align360_batch_async(r360_ctx* ctx, int n, r360_frame* const* trg, r360_frame* const* src,
                                         const float* init, int method, const r360_icp_params* p) {
    if (ctx && bind_device(ctx->device)) return -1;
    return align360_batch_enqueue(ctx, n, trg, src, init, method, p, true);
}

// wait_frames = false: the caller has already ordered ctx's stream after the frames' builds (dense queue)
int align360_batch_enqueue(r360_ctx* ctx, int n, r360_frame* const* trg, r360_frame* const* src, const float* init,
                           int method, const r360_icp_params* p, bool wait_frames) {
    CHECK_ARG(ctx && trg && src && init && p, "null arg");
    CHECK_ARG(n >= 1 && n <= R360_MAX_BATCH, "batch size must be 1..R360_MAX_BATCH");
    CHECK_ARG(!ctx->batch_pending, "a batch is pending on this ctx (r360_align360_batch_result)");
    CHECK_ARG(method >= 0 && method <= 2, "invalid method");
    for (int j = 0; j < n; ++j) {
        if (int rc = check_pair(ctx, trg[j], src[j], p)) return rc;
        CHECK_ARG(src[j]->sph_rows == src[0]->sph_rows && src[j]->sph_cols == src[0]->sph_cols,
                  "batched alignments need frames of one sphere size");
    }
    if (ensure_batch(ctx, n, (long)src[0]->lv[0].rows * src[0]->lv[0].cols)) return -1;
    std::vector<r360_frame*> fr;
    for (int j = 0; j < n; ++j) { fr.push_back(trg[j]); fr.push_back(src[j]); }
    if (wait_frames && ctx_wait_frames(ctx, fr.data(), 2 * n)) return -1;
    for (int j = 0; j < n; ++j) {
        IcpState* h = ctx->h_bstate + j;
        memset(h, 0, sizeof(IcpState));
        memcpy(h->pose, init + 16 * j, sizeof(float) * 16);
        memcpy(h->cand, init + 16 * j, sizeof(float) * 16);
        h->dbg[8] = ~0ull;
    }
    R360_HIP(hipMemcpyAsync(ctx->d_bstate, ctx->h_bstate, sizeof(IcpState) * n, hipMemcpyHostToDevice, ctx->stream));
    const size_t tk = (size_t)R360_TICKET_GROUPS * R360_TICKET_STRIDE;
    for (int l = p->n_pyr - 1; l >= 0; --l) {
        IcpJobs jobs;
        for (int j = 0; j < n; ++j) {
            IcpJob& J = jobs.j[j];
            J.src = src[j]->lv[l].p0; J.trg = trg[j]->lv[l].p0; J.tg = trg[j]->lv[l].tg;
            J.pts = src[j]->lv[l].pts; J.npts = src[j]->d_npts + l;
            J.spk = src[j]->lv[l].pk; J.tpk = trg[j]->lv[l].pk;
            J.S = ctx->d_bstate + j;
            J.partials = ctx->d_bpartials + (size_t)j * 32 * ctx->partials_cap;
            J.gcnt = ctx->d_bgticket + (size_t)j * tk;
            J.dq = ctx->d_bdefer + (size_t)j * ctx->bdefer_cap;
        }
        const int np = src[0]->lv[l].rows * src[0]->lv[l].cols;
        const IcpConst C = make_const(p, l, np, 0);
        const int passes = 1 + ((l == 0 && p->fixed_iters_level0 > 0) ? p->fixed_iters_level0 : p->max_iters);
        // the coarse levels as one persistent launch each (k_icp_levels_batch); level 0 pass by pass
        const int prc = launch_icp_levels_batch(ctx, jobs, n, src[0], l, method, C, passes);
        if (prc < 0) return prc;
        if (prc == 0) continue;
        for (int k = 0; k < passes; ++k)
            if (int rc = launch_icp_jobs(ctx, jobs, n, src[0], l, method, C, k == 0, 0)) return rc;
    }
    ctx->batch_n = n;
    ctx->batch_pending = 1;
    return 0;
}

extern "C" int r360_align360_batch_result(r360_ctx* ctx, float* pose_out, float* H_out, float* g_out,
                                          r360_icp_stats* st) {
    CHECK_ARG(ctx && ctx->batch_pending, "no batched alignment pending");
    const int n = ctx->batch_n;
    R360_HIP(hipMemcpyAsync(ctx->h_bstate, ctx->d_bstate, sizeof(IcpState) * n, hipMemcpyDeviceToHost, ctx->stream));
    if (ctx_wait(ctx)) return -1;
    ctx->batch_pending = 0;
    bool fault = false;
    for (int j = 0; j < n; ++j) fault = fault || ctx->h_bstate[j].fault;
    if (fault) {
        // a persistent coarse-level launch timed out on a job's hand-off: its drained grid left group arrival counters
        // part-way (only a pass's step workgroup resets them); zero every job's for the next batch on this ctx
        R360_HIP(hipMemsetAsync(ctx->d_bgticket, 0, sizeof(unsigned) * R360_TICKET_STRIDE * R360_TICKET_GROUPS * n,
                                ctx->stream));
        R360_HIP(hipStreamSynchronize(ctx->stream));
        r360_set_error("alignFrames360 batch: a persistent level launch timed out waiting for a pass (GPU oversubscribed?)");
        return -1;
    }
    int ill = 0;
    for (int j = 0; j < n; ++j) {
        const IcpState* h = ctx->h_bstate + j;
        if (pose_out) memcpy(pose_out + 16 * j, h->pose, sizeof(float) * 16);
        if (H_out) memcpy(H_out + 36 * j, h->Hout, sizeof(float) * 36);
        if (g_out) memcpy(g_out + 6 * j, h->gout, sizeof(float) * 6);
        if (st) fill_stats(h, st + j);
        ill += h->illposed ? 1 : 0;
    }
    return ill;
}

// one eval-mode pass (no GN step): the raw pass sums at `pose`
static int icp_eval_sums(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int level, const float pose[16], int method,
                         int occ, const r360_icp_params* p, double sums[R360_NSUMS]) {
    if (int rc = check_pair(ctx, trg, src, p)) return rc;
    CHECK_ARG(level >= 0 && level < src->n_levels, "level out of range");
    CHECK_ARG(method >= 0 && method <= 2, "invalid method");
    CHECK_ARG(occ >= 0 && occ <= 2, "occlusion must be 0, 1 or 2");
    if (ensure_defer(ctx, src->lv[level].rows * src->lv[level].cols)) return -1;
    IcpState* h = ctx->h_state;
    memset(h, 0, sizeof(IcpState));
    memcpy(h->cand, pose, sizeof(float) * 16);
    memcpy(h->pose, pose, sizeof(float) * 16);
    h->dbg[8] = ~0ull;
    R360_HIP(hipMemcpyAsync(ctx->d_state, h, sizeof(IcpState), hipMemcpyHostToDevice, ctx->stream));
    const IcpConst C = make_const(p, level, src->lv[level].rows * src->lv[level].cols, occ);
    if (launch_icp_level(ctx, trg, src, level, method, C, 0, 1)) return -1;
    R360_HIP(hipMemcpyAsync(h, ctx->d_state, sizeof(IcpState), hipMemcpyDeviceToHost, ctx->stream));
    if (ctx_wait(ctx)) return -1;
    memcpy(sums, h->sums, sizeof(double) * R360_NSUMS);
    return 0;
}

static void sums_hg(const double* s, double H[36], double g[6]) {
    int k = 0;
    for (int u = 0; u < 6; ++u)
        for (int v = u; v < 6; ++v) { H[u * 6 + v] = H[v * 6 + u] = s[k++]; }
    for (int u = 0; u < 6; ++u) g[u] = s[21 + u];
}

extern "C" int r360_icp_eval(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int level, const float pose[16],
                             int method, const r360_icp_params* p, double H[36], double g[6], double* err2,
                             int* n_valid, int* n_visible) {
    double s[R360_NSUMS];
    if (int rc = icp_eval_sums(ctx, trg, src, level, pose, method, 0, p, s)) return rc;
    sums_hg(s, H, g);
    if (err2) *err2 = s[R360_SUM_ERR2];
    if (n_valid) *n_valid = (int)s[R360_SUM_NVALID];
    if (n_visible) *n_visible = (int)s[R360_SUM_NVIS];
    return 0;
}

extern "C" int r360_icp_eval_occ(r360_ctx* ctx, r360_frame* trg, r360_frame* src, int level, const float pose[16],
                                 int method, int occlusion, const r360_icp_params* p, double H[36], double g[6],
                                 double* error, int* n_valid, int* n_visible) {
    double s[R360_NSUMS];
    if (int rc = icp_eval_sums(ctx, trg, src, level, pose, method, occlusion, p, s)) return rc;
    sums_hg(s, H, g);
    const double e2 = s[R360_SUM_ERR2], nv = s[R360_SUM_NVALID];
    if (error)
        *error = occlusion == 0 ? std::sqrt(e2 / nv)
               : occlusion == 1 ? std::sqrt(e2 / nv) + std::sqrt(s[R360_SUM_ERR2D] / s[R360_SUM_NDEPTH])
                                : std::sqrt(e2 / nv) + std::sqrt(s[R360_SUM_ERR2D] / nv);
    if (n_valid) *n_valid = (int)(nv + (occlusion == 1 ? s[R360_SUM_NDEPTH] : 0.0));
    if (n_visible) *n_visible = (int)s[R360_SUM_NVIS];
    return 0;
}

// CPose3D::exp (host copy for callers of the façade, e.g. the Register() alias)
extern "C" void r360_exp_se3(const double mu[6], int pseudo, float T[16]) {
    const double wx = mu[3], wy = mu[4], wz = mu[5];
    const double th2 = wx * wx + wy * wy + wz * wz, th = std::sqrt(th2);
    double A, B, Cc;
    if (th < 1e-6) { A = 1 - th2 / 6; B = 0.5 - th2 / 24; Cc = 1.0 / 6 - th2 / 120; }
    else { A = std::sin(th) / th; B = (1 - std::cos(th)) / th2; Cc = (th - std::sin(th)) / (th2 * th); }
    const double W[9] = {0, -wz, wy, wz, 0, -wx, -wy, wx, 0};
    double W2[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += W[r * 3 + k] * W[k * 3 + c];
            W2[r * 3 + c] = s;
        }
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) {
            double v;
            const double I = (r == c) ? 1.0 : 0.0;
            if (r < 3 && c < 3) v = I + A * W[r * 3 + c] + B * W2[r * 3 + c];
            else if (r < 3) {
                if (pseudo) v = mu[r];
                else {
                    v = 0;
                    for (int k = 0; k < 3; ++k) v += ((r == k ? 1.0 : 0.0) + B * W[r * 3 + k] + Cc * W2[r * 3 + k]) * mu[k];
                }
            } else v = (c == 3) ? 1.0 : 0.0;
            T[c * 4 + r] = (float)v;
        }
}

// Diagnostic: the s_memrealtime stamps of the last pass (only written by a -DR360_STAMPS build).
extern "C" int r360_ctx_debug_stamps(r360_ctx* ctx, unsigned long long* out12) {
    CHECK_ARG(ctx && out12, "null arg");
    R360_HIP(hipStreamSynchronize(ctx->stream));
    R360_HIP(hipMemcpy(out12, (const char*)ctx->d_state + offsetof(IcpState, dbg), sizeof(unsigned long long) * 12,
                       hipMemcpyDeviceToHost));
    return 0;
}
