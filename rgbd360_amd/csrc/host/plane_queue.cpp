// plane_queue.cpp — the plane stage of many frames, batched on one stream.
//
// Frame360::getPlanes (Frame360.h:615-640, 942-1081) per frame is a chain of ~35 kernels whose longest links
// (the boundary trace, the refinement sweeps, the plane fit) are one workgroup per sensor.  With every pipeline
// running its frames' chains on its own stream, those streams share the few pooled hardware queues (in-order
// packets): a frame's chain waited behind the other pipelines' kernels, 5.4 ms per frame under load against 0.81 ms
// alone (profiles/r5_queues).  Here the pipelines' frames go to one queue: a dispatcher thread takes every frame
// waiting (up to max_batch of one size) and launches the chain ONCE for all of them (PlaneBatch: kernel grid z = the
// frames), so a batch of F frames costs one chain of launches and its one-workgroup-per-sensor kernels run F x 8
// workgroups side by side.  The queue has two streams, each with a hardware queue of its own (CU-masked streams): a
// batch goes to the stream whose previous batch has finished, so the latency-bound chains of two batches overlap.
// Each frame keeps its own buffers and host assembly; its results equal its lone build's bit for bit (the
// kernels are the same and every frame's arithmetic is independent of the others').
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include "../r360_internal.h"

struct PlaneTicket {
    std::mutex m;
    std::condition_variable cv;
    bool enqueued = false;   // the batch's kernels and the frame's `done` event are on the queue's stream
    int rc = 0;
    std::string err;
};

struct r360_plane_queue {
    r360_ctx* ctx = nullptr;   // the queue's first stream (and per-launch timing)
    int max_batch = R360_PLANE_BATCH;
    // the queue's streams (each with a hardware queue of its own): batches go to the stream whose previous batch
    // has finished, so the latency-bound chains of two batches can overlap; stream k's batches use vox[k]
    std::vector<hipStream_t> streams;
    std::vector<std::vector<VoxSlot>> vox;   // voxel-fallback scratch per stream and batch slot
    std::vector<hipEvent_t> last;            // per stream: the end of its last batch (nullptr: none yet)
    struct Item { r360_frame* f; std::shared_ptr<PlaneTicket> tk; };
    std::deque<Item> pending;
    std::mutex m;
    std::condition_variable cv;
    bool quit = false;
    std::thread worker;
    long batches = 0, frames = 0;
    int max_seen = 0;
};

int planes_launch(const PlaneBatch& B, int F, const PlaneGeom& G, hipStream_t st, r360_ctx* tctx,
                  const hipEvent_t* bgr_ev);   // pbmap.cpp

namespace {

bool same_geom(const PlaneGeom& a, const PlaneGeom& b) {
    return a.rows == b.rows && a.cols == b.cols && a.w == b.w && a.h == b.h && a.sd_max == b.sd_max &&
           a.grid_cells == b.grid_cells;
}

void dispatcher(r360_plane_queue* q) {
    (void)hipSetDevice(q->ctx->device);
    const int ns = (int)q->streams.size();
    int next = 0;
    for (;;) {
        // a stream whose previous batch has finished (else wait for the one that started first): frames that
        // arrive while every stream is busy go into the next launch
        int k = -1;
        for (int t = 0; t < ns && k < 0; ++t) {
            const int c = (next + t) % ns;
            if (!q->last[c] || hipEventQuery(q->last[c]) == hipSuccess) k = c;
        }
        if (k < 0) {
            k = next;
            (void)event_wait(q->last[k]);
        }
        next = (k + 1) % ns;
        std::vector<r360_plane_queue::Item> take;
        {
            std::unique_lock<std::mutex> lk(q->m);
            q->cv.wait(lk, [&] { return q->quit || !q->pending.empty(); });
            if (q->pending.empty()) return;   // quit with nothing pending
            const PlaneGeom G0 = plane_geom(q->pending.front().f);
            for (auto it = q->pending.begin(); it != q->pending.end() && (int)take.size() < q->max_batch;) {
                if (same_geom(plane_geom(it->f), G0)) { take.push_back(*it); it = q->pending.erase(it); }
                else ++it;
            }
        }
        const int F = (int)take.size();
        const PlaneGeom G = plane_geom(take[0].f);
        hipStream_t st = q->streams[k];
        int rc = 0;
        PlaneBatch B;
        std::memset(&B, 0, sizeof B);
        for (int j = 0; j < F && rc == 0; ++j) {
            r360_frame* f = take[j].f;
            rc = vox_slot_reserve(q->vox[k][j], G, st);
            if (rc == 0 && hipStreamWaitEvent(st, f->pl.ready, 0) != hipSuccess) {
                r360_set_error("plane queue: hipStreamWaitEvent failed");
                rc = -1;
            }
            B.f[j] = plane_dev(f, q->vox[k][j].v);
        }
        // per-launch timing (r360_ctx_timing) records on the ctx's stream: the first stream's batches only
        hipEvent_t bev[R360_PLANE_BATCH] = {};
        for (int j = 0; j < F; ++j) bev[j] = take[j].f->bgr_wait();
        if (rc == 0) rc = planes_launch(B, F, G, st, k == 0 ? q->ctx : nullptr, bev);
        for (int j = 0; j < F && rc == 0; ++j)
            if (hipEventRecord(take[j].f->pl.done, st) != hipSuccess) {
                r360_set_error("plane queue: hipEventRecord failed");
                rc = -1;
            }
        if (rc == 0) {
            if (!q->last[k] && hipEventCreateWithFlags(&q->last[k], hipEventDisableTiming) != hipSuccess) q->last[k] = nullptr;
            if (q->last[k] && hipEventRecord(q->last[k], st) != hipSuccess) {
                hipEventDestroy(q->last[k]);
                q->last[k] = nullptr;
            }
        }
        const std::string err = rc ? r360_last_error() : std::string();
        for (auto& it : take) {
            std::lock_guard<std::mutex> lk(it.tk->m);
            it.tk->rc = rc;
            it.tk->err = err;
            it.tk->enqueued = true;
            it.tk->cv.notify_all();
        }
        std::lock_guard<std::mutex> lk(q->m);
        ++q->batches;
        q->frames += F;
        if (F > q->max_seen) q->max_seen = F;
    }
}

}  // namespace

int plane_queue_create(int device, int max_batch, r360_plane_queue** out) {
    // experiment builds: R360_PLANE_STREAMS streams (default 2)
    static const int nstreams = R360_KNOB("R360_PLANE_STREAMS", 2);
    CHECK_ARG(out && max_batch >= 1 && max_batch <= R360_PLANE_BATCH, "plane queue: max_batch must be 1..8");
    r360_ctx* ctx = nullptr;
    if (int rc = r360_ctx_create(device, &ctx)) return rc;
    // hardware queues of their own: a stream with a CU mask (all CUs) is not put in the pooled queues
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
        r360_set_error("plane queue: hipDeviceGetAttribute failed");
        r360_ctx_destroy(ctx);
        return -1;
    }
    uint32_t mask[R360_CU_MASK_WORDS] = {0};
    for (int i = 0; i < cus && i < 32 * R360_CU_MASK_WORDS; ++i) mask[i / 32] |= 1u << (i % 32);
    auto* q = new r360_plane_queue;
    q->ctx = ctx;
    q->max_batch = max_batch;
    const int ns = nstreams >= 1 && nstreams <= 4 ? nstreams : 1;
    // experiment builds: R360_PLANE_PRIO=1 / 2 gives the streams the device's highest / lowest priority instead of
    // a CU mask (a priority stream also gets a hardware queue of its own)
    static const int prio = R360_KNOB("R360_PLANE_PRIO", 0);
    for (int k = 0; k < ns; ++k) {
        hipStream_t hs = nullptr;
        if (prio) {
            int least = 0, greatest = 0;
            if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
                hipStreamCreateWithPriority(&hs, hipStreamNonBlocking, prio == 1 ? greatest : least) != hipSuccess)
                hs = nullptr;
        } else if (hipExtStreamCreateWithCUMask(&hs, R360_CU_MASK_WORDS * 32, mask) != hipSuccess) {
            hs = nullptr;
        }
        if (!hs) {
            r360_set_error("plane queue: stream creation failed");
            for (hipStream_t t : q->streams) hipStreamDestroy(t);
            r360_ctx_destroy(ctx);
            delete q;
            return -1;
        }
        q->streams.push_back(hs);
    }
    // the ctx's own stream is replaced by the first CU-masked one (nothing was enqueued on it yet)
    if (hipStreamSynchronize(ctx->stream) != hipSuccess || hipStreamDestroy(ctx->stream) != hipSuccess) {
        r360_set_error("plane queue: releasing the context's stream failed");
        for (hipStream_t t : q->streams) hipStreamDestroy(t);
        ctx->stream_borrowed = true;   // already released
        r360_ctx_destroy(ctx);
        delete q;
        return -1;
    }
    ctx->stream = q->streams[0];
    q->vox.assign(ns, std::vector<VoxSlot>(max_batch));
    q->last.assign(ns, nullptr);
    q->worker = std::thread(dispatcher, q);
    *out = q;
    return 0;
}

void plane_queue_destroy(r360_plane_queue* q) {
    if (!q) return;
    {
        std::lock_guard<std::mutex> lk(q->m);
        q->quit = true;
    }
    q->cv.notify_all();
    q->worker.join();
    (void)hipSetDevice(q->ctx->device);
    for (hipStream_t st : q->streams) (void)hipStreamSynchronize(st);
    for (auto& vs : q->vox)
        for (auto& v : vs) vox_slot_free(v);
    for (hipEvent_t e : q->last)
        if (e) hipEventDestroy(e);
    for (size_t k = 1; k < q->streams.size(); ++k) hipStreamDestroy(q->streams[k]);
    r360_ctx_destroy(q->ctx);   // destroys streams[0] (the ctx's stream)
    delete q;
}

r360_ctx* plane_queue_ctx(r360_plane_queue* q) { return q ? q->ctx : nullptr; }

// every stream's batch slots' voxel scratch sized for frames of G now (before any frame is submitted)
int plane_queue_reserve(r360_plane_queue* q, const PlaneGeom& G) {
    for (size_t k = 0; k < q->streams.size(); ++k)
        for (auto& v : q->vox[k])
            if (vox_slot_reserve(v, G, q->streams[k])) return -1;
    R360_HIP(hipDeviceSynchronize());
    return 0;
}

int plane_queue_stats(const r360_plane_queue* q, long* batches, long* frames, int* max_batch_seen) {
    CHECK_ARG(q, "null plane queue");
    auto* mq = const_cast<r360_plane_queue*>(q);
    std::lock_guard<std::mutex> lk(mq->m);
    if (batches) *batches = q->batches;
    if (frames) *frames = q->frames;
    if (max_batch_seen) *max_batch_seen = q->max_seen;
    return 0;
}

// The frame's inputs (upload, undistort) are enqueued on its own stream: its ready event marks their end, and the
// queue's stream waits on it.  The frame's ticket tells the assembly pool when `done` has been recorded.
int plane_queue_submit(r360_plane_queue* q, r360_frame* f) {
    CHECK_ARG(q && f, "null arg");
    PlaneBufs& P = f->pl;
    R360_HIP(hipEventRecord(P.ready, f->ctx->stream));
    auto tk = std::make_shared<PlaneTicket>();
    P.ticket = tk;
    {
        std::lock_guard<std::mutex> lk(q->m);
        q->pending.push_back(r360_plane_queue::Item{f, tk});
    }
    q->cv.notify_one();
    return 0;
}

// the frame's batch state for the host assembly pool (host/pbmap.cpp): whether `done` has been recorded
int plane_ticket_poll(const std::shared_ptr<PlaneTicket>& tk, std::string* err) {
    std::lock_guard<std::mutex> lk(tk->m);
    if (!tk->enqueued) return 0;
    if (tk->rc) {
        if (err) *err = tk->err;
        return -1;
    }
    return 1;
}
