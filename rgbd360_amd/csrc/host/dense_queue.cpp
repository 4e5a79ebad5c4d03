#include <cstdlib>
// dense_queue.cpp — the dense stage of many concurrent registrations, batched on one stream.
//
// OdometryRGBD360 registers every consecutive pair (OdometryRGBD360.cpp:141-257), and SphereGraphSLAM /
// LoopClosure360 register a frame against several keyframes; each registration ends in one alignFrames360
// (RegisterPhotoICP.h:4519-4784).  Producers (pipelines of frame builds + PbMap stages, one host thread each)
// submit their alignments here; a dispatcher thread takes every pending alignment (up to R360_MAX_BATCH of
// one method / parameter set) and runs them as ONE batched alignment (r360_align360_batch_async): one launch
// per pass over all pairs instead of one small launch per pair and stream.  While a batch runs, the next one
// accumulates, so the batch size follows the load.  A job's result is exactly the single-pair result.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include "../r360_internal.h"

extern "C" int r360_align360_batch_async(r360_ctx* ctx, int n, r360_frame* const* trg, r360_frame* const* src,
                                         const float* init, int method, const r360_icp_params* p);
int align360_batch_enqueue(r360_ctx* ctx, int n, r360_frame* const* trg, r360_frame* const* src, const float* init,
                           int method, const r360_icp_params* p, bool wait_frames);
hipEvent_t frame_build_event(const r360_frame* f);   // runtime.cpp: recorded after the frame's last pyramid build

struct r360_dense_queue {
    r360_ctx* ctx = nullptr;           // the queue's own stream, GN states and batch buffers
    // Batches in flight: up to n_ctx at once, batch k on cx[k % n_ctx]'s stream.  The dispatcher enqueues a batch
    // as soon as jobs are pending and a stream is free; the collector thread reads results in batch order.  With
    // one stream the next batch could only be enqueued after the previous one's result was read (a host round
    // trip plus ~65 launches' enqueue per batch with the dense stream idle), and every pass's tail (ticket, GN step)
    // left the GPU to the other streams alone.
    r360_ctx* cx[2] = {nullptr, nullptr};
    int n_ctx = 1;
    bool busy[2] = {false, false};
    bool split = false;   // each batch split over both streams (the halves' passes interleave on the GPU)
    struct Inflight {
        int slot = 0, n = 0, rc = 0;
        int n0 = 0;       // split batch: jobs [0, n0) on cx[0], [n0, n) on cx[1]
        std::vector<long> take;
        std::string err;
    };
    std::deque<Inflight> inflight;
    bool dispatch_done = false;
    std::thread collector;
    std::condition_variable cv_flight;
    int max_batch = R360_MAX_BATCH;
    std::mutex m;
    std::condition_variable cv_work, cv_done;
    struct Job {
        r360_frame* trg = nullptr;
        r360_frame* src = nullptr;
        float init[16];
        int method = 0;
        r360_icp_params p{};
        hipEvent_t ev[2] = {nullptr, nullptr};   // the frames' builds (their build events, or the streams at submit)
        bool own[2] = {false, false};            // ev[e] came from ev_free (the frames' build events are not ours)
        unsigned gen[2] = {0, 0};                // the frames' build generations when ev[e] was their build event
        int nev = 0;
        int reg = 0, good = 0;                   // Register(): PbMap outcome and information
        float info[36];
        int done = 0, rc = 0;
        bool claimed = false;                    // a collector waits on it (a second one is refused)
        std::string err;
        float pose[16], H[36], g[6];
        r360_icp_stats st{};
    };
    std::map<long, Job> jobs;
    std::deque<long> pending;
    long next = 1;
    bool quit = false;
    std::thread worker;
    std::vector<hipEvent_t> ev_free;
    long batches = 0, batched = 0;
    int max_seen = 0;
};

// One batch = one method, one parameter set and one sphere geometry (r360_align360_batch_async rejects a
// batch whose frames differ in size, which would fail every job of it)
static bool same_params(const r360_dense_queue::Job& a, const r360_dense_queue::Job& b) {
    return a.method == b.method && memcmp(&a.p, &b.p, sizeof(r360_icp_params)) == 0 &&
           a.src->sph_rows == b.src->sph_rows && a.src->sph_cols == b.src->sph_cols &&
           a.src->n_levels == b.src->n_levels && a.trg->n_levels == b.trg->n_levels;
}

static int free_slot(const r360_dense_queue* q) {
    for (int k = 0; k < q->n_ctx; ++k)
        if (!q->busy[k]) return k;
    return -1;
}

static void dispatcher(r360_dense_queue* q) {
    (void)hipSetDevice(q->ctx->device);
    std::vector<r360_frame*> trg, src;
    std::vector<float> init;
    for (;;) {
        std::unique_lock<std::mutex> lk(q->m);
        auto can_go = [&] { return q->split ? (!q->busy[0] && !q->busy[1]) : free_slot(q) >= 0; };
        q->cv_work.wait(lk, [&] { return (!q->pending.empty() && can_go()) || (q->quit && q->pending.empty()); });
        if (q->pending.empty()) break;   // quit with nothing pending
        // optional batch floor (R360_QUEUE_MIN jobs, waiting at most R360_QUEUE_WAIT_US): larger batches fill the
        // level-0 pass better at the cost of latency (experiment knob, off by default)
        static const int min_jobs = R360_KNOB("R360_QUEUE_MIN", 0);
        static const int wait_us = R360_KNOB("R360_QUEUE_WAIT_US", 2000);
        if (min_jobs > 1 && (int)q->pending.size() < min_jobs)
            q->cv_work.wait_for(lk, std::chrono::microseconds(wait_us),
                                [&] { return q->quit || (int)q->pending.size() >= min_jobs; });
        r360_dense_queue::Inflight b;
        b.slot = free_slot(q);
        q->busy[b.slot] = true;
        const r360_dense_queue::Job& first = q->jobs[q->pending.front()];
        for (auto it = q->pending.begin(); it != q->pending.end() && (int)b.take.size() < q->max_batch;) {
            if (same_params(q->jobs[*it], first)) { b.take.push_back(*it); it = q->pending.erase(it); }
            else ++it;
        }
        const int n = (int)b.take.size();
        b.n = n;
        b.n0 = (q->split && n >= 2) ? (n + 1) / 2 : n;
        if (b.n0 < n) { b.slot = 0; q->busy[0] = q->busy[1] = true; }
        trg.resize(n); src.resize(n); init.resize(16 * (size_t)n);
        for (int j = 0; j < n; ++j) {
            r360_dense_queue::Job& J = q->jobs[b.take[j]];
            trg[j] = J.trg; src[j] = J.src;
            memcpy(init.data() + 16 * j, J.init, sizeof J.init);
        }
        const int method = first.method;
        const r360_icp_params p = first.p;
        std::vector<hipEvent_t> evs;
        int rc = 0;
        for (long t : b.take) {
            const r360_dense_queue::Job& J = q->jobs[t];
            for (int e = 0; e < J.nev; ++e) {
                evs.push_back(J.ev[e]);
                // a frame's build event is re-recorded by every rebuild: the job's frames must not have been
                // rebuilt between its submit and this dispatch (the callers collect a pair before refilling its
                // buffers), or the batch would wait on the wrong build
                const r360_frame* f = e == 0 ? J.trg : J.src;
                if (!J.own[e] && f->build_gen.load(std::memory_order_acquire) != J.gen[e]) {
                    r360_set_error("dense queue: a frame was rebuilt while its alignment was pending");
                    rc = -1;
                }
            }
        }
        lk.unlock();

        for (int part = 0; part < (b.n0 < n ? 2 : 1) && rc == 0; ++part) {
            r360_ctx* c = q->cx[part ? 1 : b.slot];
            const int j0 = part ? b.n0 : 0, nj = part ? n - b.n0 : b.n0;
            for (hipEvent_t e : evs)
                if (hipStreamWaitEvent(c->stream, e, 0) != hipSuccess) { r360_set_error("hipStreamWaitEvent failed"); rc = -1; }
            if (rc == 0)
                rc = align360_batch_enqueue(c, nj, trg.data() + j0, src.data() + j0, init.data() + 16 * j0, method, &p, false);
        }
        b.rc = rc;
        if (rc < 0) b.err = r360_last_error();

        lk.lock();
        q->inflight.push_back(std::move(b));
        lk.unlock();
        q->cv_flight.notify_one();
    }
    {
        std::lock_guard<std::mutex> lk(q->m);
        q->dispatch_done = true;
    }
    q->cv_flight.notify_one();
}

// Reads the batches' results in enqueue order and hands them to the waiting collectors.
static void collector(r360_dense_queue* q) {
    (void)hipSetDevice(q->ctx->device);
    for (;;) {
        std::unique_lock<std::mutex> lk(q->m);
        q->cv_flight.wait(lk, [&] { return q->dispatch_done || !q->inflight.empty(); });
        if (q->inflight.empty()) break;   // dispatcher gone, nothing left
        r360_dense_queue::Inflight b = q->inflight.front();
        lk.unlock();

        const int n = b.n;
        std::vector<float> po(16 * (size_t)n), Ho(36 * (size_t)n), go(6 * (size_t)n);
        std::vector<r360_icp_stats> st(n);
        int rc = b.rc;
        std::string err = b.err;
        if (rc == 0) {
            rc = r360_align360_batch_result(q->cx[b.slot], po.data(), Ho.data(), go.data(), st.data());
            if (rc >= 0 && b.n0 < n) {
                const int j0 = b.n0;
                rc = r360_align360_batch_result(q->cx[1], po.data() + 16 * j0, Ho.data() + 36 * j0, go.data() + 6 * j0,
                                                st.data() + j0);
            }
            if (rc < 0) err = r360_last_error();
        }

        lk.lock();
        for (int j = 0; j < n; ++j) {
            r360_dense_queue::Job& J = q->jobs[b.take[j]];
            if (rc < 0) { J.rc = rc; J.err = err; }
            else {
                memcpy(J.pose, po.data() + 16 * j, sizeof J.pose);
                memcpy(J.H, Ho.data() + 36 * j, sizeof J.H);
                memcpy(J.g, go.data() + 6 * j, sizeof J.g);
                J.st = st[j];
                J.rc = st[j].illposed ? 1 : 0;
            }
            for (int e = 0; e < J.nev; ++e)
                if (J.own[e]) q->ev_free.push_back(J.ev[e]);
            J.nev = 0;
            J.done = 1;
        }
        q->batches++;
        q->batched += n;
        if (n > q->max_seen) q->max_seen = n;
        q->inflight.pop_front();
        q->busy[b.slot] = false;
        if (b.n0 < n) q->busy[1] = false;
        lk.unlock();
        q->cv_done.notify_all();
        q->cv_work.notify_one();
    }
}

extern "C" int r360_dense_queue_create(int device, int max_batch, r360_dense_queue** out) {
    CHECK_ARG(out, "null out");
    CHECK_ARG(max_batch >= 1 && max_batch <= R360_MAX_BATCH, "max_batch must be 1..R360_MAX_BATCH_ALIGN");
    r360_ctx* ctx = nullptr;
    if (int rc = r360_ctx_create(device, &ctx)) return rc;
    // stream priority experiments (off by default): R360_QUEUE_PRIORITY=1 puts the queue's stream at the device's
    // highest priority (batched passes dispatched ahead of the plane kernels: 603 vs 820 pairs/s, the plane half
    // starves); with R360_CTX_PRIORITY=1 (pipelines high) the queue stays at the normal priority
    static const int prio_env = R360_KNOB("R360_QUEUE_PRIORITY", 0);
    static const int ctx_prio = R360_KNOB("R360_CTX_PRIORITY", 0);
    if (prio_env != 0 || ctx_prio != 0) {
        int least = 0, greatest = 0;
        R360_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        hipStream_t hs = nullptr;
        // R360_QUEUE_PRIORITY=2: the queue's stream at the lowest priority (its own hardware queue), pipelines normal
        R360_HIP(hipStreamCreateWithPriority(&hs, hipStreamNonBlocking, prio_env == 1 ? greatest : least));
        R360_HIP(hipStreamDestroy(ctx->stream));
        ctx->stream = hs;
    }
    uint32_t mask[R360_CU_MASK_WORDS];
    // The queue's stream on a hardware queue of its own (a stream with a CU mask, here every CU, gets a dedicated HSA
    // queue outside the pool of GPU_MAX_HW_QUEUES that plain streams share).  In the pooled queues, whose packets run
    // in order, the batches waited behind the plane kernels of whichever pipelines shared their queue, and which ones
    // did depended on stream creation and first use: 1240-1250 vs 1320-1335 pairs/s with its own queue, in one session
    // (profiles/r5_queues).  R360_QUEUE_OWNQ=0 (experiment builds) leaves it in the pool.
    static const int ownq = R360_KNOB("R360_QUEUE_OWNQ", 1);
    if (ownq && prio_env == 0 && ctx_prio == 0) {
        int cus = 0;
        R360_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        for (int w = 0; w < R360_CU_MASK_WORDS; ++w) mask[w] = 0;
        for (int i = 0; i < cus && i < 32 * R360_CU_MASK_WORDS; ++i) mask[i / 32] |= 1u << (i % 32);
        hipStream_t hs = nullptr;
        R360_HIP(hipExtStreamCreateWithCUMask(&hs, R360_CU_MASK_WORDS * 32, mask));
        R360_HIP(hipStreamDestroy(ctx->stream));
        ctx->stream = hs;
    } else if (r360_cu_mask(device, 1, mask)) {   // CU partition experiment: the queue's stream off the excluded CUs
        hipStream_t hs = nullptr;
        R360_HIP(hipExtStreamCreateWithCUMask(&hs, R360_CU_MASK_WORDS * 32, mask));
        R360_HIP(hipStreamDestroy(ctx->stream));
        ctx->stream = hs;
    }
    auto* q = new r360_dense_queue;
    q->ctx = ctx;
    q->cx[0] = ctx;
    // one batch stream; R360_QUEUE_STREAMS=2 (experiment builds) alternates batches over two: measured slower
    // (1206-1227 vs 1263 pairs/s, profiles/r4_queue): the batches halve (4.1 vs 7.7 pairs per launch)
    static const int streams = R360_KNOB("R360_QUEUE_STREAMS", 1);
    // R360_QUEUE_SPLIT=1 (experiment builds): one batch at a time, its jobs split over the two streams
    static const int split = R360_KNOB("R360_QUEUE_SPLIT", 0);
    if (streams >= 2 || split) {
        r360_ctx* c2 = nullptr;
        if (int rc = r360_ctx_create(device, &c2)) {
            r360_ctx_destroy(ctx);
            delete q;
            return rc;
        }
        q->cx[1] = c2;
        q->n_ctx = 2;
        q->split = split != 0;
        ctx->stats_sibling = c2;   // kernel statistics of the queue ctx cover both streams
    }
    q->max_batch = max_batch;
    q->worker = std::thread(dispatcher, q);
    q->collector = std::thread(collector, q);
    *out = q;
    return 0;
}

// Sizes the queue's batch buffers for its largest batch of frames of n_pixels level-0 pixels now (before any job:
// ensure_batch synchronises the device when it grows a buffer, which a first large batch would otherwise do mid-run)
int dense_queue_reserve(r360_dense_queue* q, long n_pixels) {
    for (int k = 0; k < q->n_ctx; ++k)
        if (ensure_batch(q->cx[k], q->max_batch, n_pixels)) return -1;
    return 0;
}

extern "C" void r360_dense_queue_destroy(r360_dense_queue* q) {
    if (!q) return;
    {
        std::lock_guard<std::mutex> lk(q->m);
        q->quit = true;
    }
    q->cv_work.notify_all();
    q->worker.join();
    q->collector.join();
    (void)hipSetDevice(q->ctx->device);
    for (auto& kv : q->jobs)
        for (int e = 0; e < kv.second.nev; ++e)
            if (kv.second.own[e]) hipEventDestroy(kv.second.ev[e]);
    for (hipEvent_t e : q->ev_free) hipEventDestroy(e);
    q->ctx->stats_sibling = nullptr;
    if (q->cx[1]) r360_ctx_destroy(q->cx[1]);
    r360_ctx_destroy(q->ctx);
    delete q;
}

extern "C" r360_ctx* r360_dense_queue_ctx(r360_dense_queue* q) { return q ? q->ctx : nullptr; }

extern "C" int r360_dense_queue_stats(r360_dense_queue* q, long* batches, long* jobs, int* max_batch_seen) {
    CHECK_ARG(q, "null queue");
    std::lock_guard<std::mutex> lk(q->m);
    if (batches) *batches = q->batches;
    if (jobs) *jobs = q->batched;
    if (max_batch_seen) *max_batch_seen = q->max_seen;
    return 0;
}

static int queue_submit(r360_dense_queue* q, r360_frame* trg, r360_frame* src, const float init[16], int method,
                        const r360_icp_params* p, int reg, int good, const float* info, long* ticket) {
    CHECK_ARG(q && trg && src && init && p && ticket, "null arg");
    CHECK_ARG(method >= 0 && method <= 2, "invalid method");
    CHECK_ARG(trg->ctx->device == q->ctx->device && src->ctx->device == q->ctx->device,
              "frames and queue on different devices");
    CHECK_ARG((trg->built & R360_BUILD_PYRAMID) && (src->built & R360_BUILD_PYRAMID),
              "frames need R360_BUILD_PYRAMID");
    // what the batch waits for: each frame's build event (recorded right after its pyramid build), or, for a frame
    // built without one, an event on its stream now (everything enqueued there so far)
    const r360_frame* fs[2] = {trg, src};
    const int ns = trg == src ? 1 : 2;
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool own[2] = {false, false};
    unsigned gen[2] = {0, 0};
    for (int i = 0; i < ns; ++i) {
        gen[i] = fs[i]->build_gen.load(std::memory_order_acquire);
        ev[i] = frame_build_event(fs[i]);
    }
    {
        std::lock_guard<std::mutex> lk(q->m);
        for (int i = 0; i < ns; ++i)
            if (!ev[i] && !q->ev_free.empty()) { ev[i] = q->ev_free.back(); q->ev_free.pop_back(); own[i] = true; }
    }
    for (int i = 0; i < ns; ++i) {
        if (!ev[i]) { R360_HIP(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming)); own[i] = true; }
        if (own[i]) R360_HIP(hipEventRecord(ev[i], fs[i]->ctx->stream));
    }
    {
        std::lock_guard<std::mutex> lk(q->m);
        const long t = q->next++;
        r360_dense_queue::Job& J = q->jobs[t];
        J.trg = trg; J.src = src;
        memcpy(J.init, init, sizeof J.init);
        J.method = method;
        J.p = *p;
        J.ev[0] = ev[0]; J.ev[1] = ev[1]; J.own[0] = own[0]; J.own[1] = own[1]; J.nev = ns;
        J.gen[0] = gen[0]; J.gen[1] = gen[1];
        J.reg = reg; J.good = good;
        if (info) memcpy(J.info, info, sizeof J.info);
        q->pending.push_back(t);
        *ticket = t;
    }
    q->cv_work.notify_one();
    return 0;
}

// waits for job t and removes it; returns its rc (0, 1 = ILL-POSED, < 0 error).  want_reg: 1 = only a
// Register() ticket, 0 = only a plain alignment ticket, -1 = either; a ticket of the other kind is left in
// the queue for the right collector.  The ticket is claimed under the lock, so a second collector of the
// same ticket is refused instead of waiting on a job the first one erases.
static int queue_collect(r360_dense_queue* q, long t, r360_dense_queue::Job& out, int want_reg = -1) {
    CHECK_ARG(q, "null queue");
    std::unique_lock<std::mutex> lk(q->m);
    auto it = q->jobs.find(t);
    CHECK_ARG(it != q->jobs.end(), "unknown or already collected ticket");
    CHECK_ARG(!it->second.claimed, "ticket is being collected by another thread");
    CHECK_ARG(want_reg < 0 || (it->second.reg != 0) == (want_reg != 0),
              want_reg ? "ticket is not a Register() job (r360_dense_queue_collect)"
                       : "ticket is a Register() job (r360_register_collect)");
    it->second.claimed = true;
    q->cv_done.wait(lk, [&] { return it->second.done != 0; });   // std::map nodes stay put while others erase
    out = it->second;
    q->jobs.erase(it);
    lk.unlock();
    if (out.rc < 0) { r360_set_error("%s", out.err.c_str()); return out.rc; }
    return out.rc;
}

extern "C" int r360_dense_queue_submit(r360_dense_queue* q, r360_frame* trg, r360_frame* src, const float init[16],
                                       int method, const r360_icp_params* p, long* ticket) {
    return queue_submit(q, trg, src, init, method, p, 0, 0, nullptr, ticket);
}

extern "C" int r360_dense_queue_collect(r360_dense_queue* q, long ticket, float pose_out[16], float H_out[36],
                                        float g_out[6], r360_icp_stats* st) {
    r360_dense_queue::Job J;
    const int rc = queue_collect(q, ticket, J, 0);
    if (rc < 0) return rc;
    if (pose_out) memcpy(pose_out, J.pose, sizeof J.pose);
    if (H_out) memcpy(H_out, J.H, sizeof J.H);
    if (g_out) memcpy(g_out, J.g, sizeof J.g);
    if (st) *st = J.st;
    return rc;
}

// Register() with the dense stage on the queue: RegisterPbMap on the calling thread (ctx's matcher), the
// rotOffset-conjugated initialisation (OdometryKeyFrame360.cpp:205-254), then the alignment is submitted.
extern "C" int r360_register_submit(r360_ctx* ctx, r360_dense_queue* q, r360_frame* ref, r360_frame* trg,
                                    const float guess[16], const r360_icp_params* p, size_t max_match_planes,
                                    int mode, long* ticket) {
    CHECK_ARG(ctx && q && ref && trg && p && ticket, "null arg");
    float pb[16], inf[36];
    for (int i = 0; i < 16; ++i) pb[i] = guess ? guess[i] : ((i % 5 == 0) ? 1.f : 0.f);
    for (int i = 0; i < 36; ++i) inf[i] = 0.f;
    const int good = r360_register_pbmap(ctx, ref, trg, max_match_planes, mode, pb, inf, nullptr, 0, nullptr, nullptr,
                                         nullptr, nullptr);
    if (good < 0) return good;
    float Ro[16], Ri[16], t1[16], init[16];
    r360_rot_offset(Ro, Ri);
    r360_mul4(Ro, pb, t1);
    r360_mul4(t1, Ri, init);                             // rotOffset * pose * rotOffset^-1
    return queue_submit(q, ref, trg, init, R360_PHOTO_DEPTH, p, 1, good, inf, ticket);
}

extern "C" int r360_register_collect(r360_dense_queue* q, long ticket, float pose[16], float info[36],
                                     r360_icp_stats* st) {
    CHECK_ARG(pose, "null pose");
    r360_dense_queue::Job J;
    const int rc = queue_collect(q, ticket, J, 1);
    if (rc < 0) return rc;
    float Ro[16], Ri[16], t2[16];
    r360_rot_offset(Ro, Ri);
    r360_mul4(Ri, J.pose, t2);
    r360_mul4(t2, Ro, pose);                             // rotOffset^-1 * dense * rotOffset
    if (info) memcpy(info, J.info, sizeof J.info);
    if (st) *st = J.st;
    return J.good ? 0 : 1;
}
