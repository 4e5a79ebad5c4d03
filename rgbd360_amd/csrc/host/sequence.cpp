// sequence.cpp — OdometryRGBD360 over a frame sequence, pipelined on one GPU (BASELINE configs[3]).
//
// The reference's loop (Registration/OdometryRGBD360.cpp:141-257) registers each new Frame360 against the previous
// one: RegisterPbMap, the rotOffset-conjugated alignFrames360 (the Register() alias, OdometryKeyFrame360.cpp:
// 205-254), and composes currentPose = currentPose * rigidTransf (:257).  Pair (i, i+1) needs only frames i and i+1.
// A call registers the pairs [p0, p1) `repeats` times; the repeats x (p1 - p0) pair registrations form one stream
// (repeat-major) that is cut into contiguous pieces, one per pipeline: a host thread of this object with its own
// r360_ctx (HIP stream, GN state, matcher scratch) and a ring of Frame360 buffers.  A piece is a list of segments
// (repeat r, pairs [a, b)); its frame positions are the segments' frames a..b back to back, and positions t, t + 1
// form a pair unless t ends a segment.  Pipelines share nothing but the dense queue: a piece builds its first frame
// (and the first frame of each later segment) itself, which costs one extra frame build per pipeline and segment
// boundary and no coupling between pipelines (runs that shared their edge frames waited on each other at every
// repeat: 1.2-1.9 ms per pair, profiles/r5_seq).
//
// Queued mode (params.queue > 0): every pipeline's alignFrames360 goes to one dense queue (r360_dense_queue, up to
// `queue` pairs per launch), and a pipeline keeps `depth` alignments in flight while it builds and PbMap-registers
// the next frames.  Frames are built `lookahead` positions ahead of the pair in hand and the next frame's upload is
// issued right after a build on the same stream.  A ring buffer is refilled only after every pair that used its
// previous frame was collected (the dense queue refuses a job whose frame was rebuilt meanwhile).
//
// Records are batch-invariant: a pair's record is bit-identical however the pairs are cut into pieces, pipelines,
// dense batches and ranks (the batched ICP grid depends on the level size only).  Against an unqueued run (each
// pair a lone Register() on its pipeline's context) the PbMap stage is identical and the dense pose equal to
// rounding (lone passes use two workgroups per CU).
#include <array>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <sys/syscall.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../r360_internal.h"

namespace {

constexpr int REC = R360_SEQ_RECORD;          // pose 16, info 36, status, SSO, error, (spare)


double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// rotOffset of OdometryRGBD360.cpp:136-139 (angle in float, PI = 3.14159265359), entries rounded to float, and the
// conjugation back to the rig frame of a dense pose, rotOffset^-1 * D * rotOffset, in double
void rig_from_dense(const float dense[16], float out[16]) {
    const double a = double(157.5f) * 3.14159265359 / 180;
    const double c = double(float(std::cos(a))), s = double(float(std::sin(a)));
    double Ro[16] = {1, 0, 0, 0, 0, c, -s, 0, 0, s, c, 0, 0, 0, 0, 1};   // column-major: (1,2) = s, (2,1) = -s
    double Ri[16] = {1, 0, 0, 0, 0, c, s, 0, 0, -s, c, 0, 0, 0, 0, 1};
    double D[16], T[16];
    for (int i = 0; i < 16; ++i) D[i] = dense[i];
    auto mul = [](const double* A, const double* B, double* Cm) {
        for (int col = 0; col < 4; ++col)
            for (int r = 0; r < 4; ++r) {
                double acc = 0;
                for (int k = 0; k < 4; ++k) acc += A[k * 4 + r] * B[col * 4 + k];
                Cm[col * 4 + r] = acc;
            }
    };
    double U[16];
    mul(Ri, D, T);
    mul(T, Ro, U);
    for (int i = 0; i < 16; ++i) out[i] = float(U[i]);
}

}  // namespace

struct r360_sequence {
    int device = 0;
    r360_sequence_params prm{};
    int P = 0;
    unsigned flags = 0;
    std::vector<r360_ctx*> ctx;
    std::vector<r360_calib*> cal;
    std::vector<std::vector<r360_frame*>> ring;   // per pipeline
    r360_dense_queue* q = nullptr;
    r360_plane_queue* pq = nullptr;               // the pipelines' plane stages, batched (plane_batch > 0)
    // persistent pipeline threads
    std::vector<std::thread> th;
    std::vector<long> tid;
    std::mutex m;
    std::condition_variable cv_go, cv_done;
    long gen = 0;
    int done = 0;
    bool quit = false;
    // the run in progress
    struct Seg { int rep, a, b; };               // pairs [a, b) of repeat rep
    struct Job {
        int p0 = 0, p1 = 0, repeats = 1, device_inputs = 0;
        std::vector<std::vector<Seg>> piece;       // per pipeline
        const void* const* bgr = nullptr;
        const void* const* dep = nullptr;
        float* out = nullptr;
    } job;
    std::vector<int> rc;
    std::vector<std::string> err;
    std::vector<std::array<double, 8>> host_s;     // per pipeline: see r360_sequence_host_times
};

namespace {

struct Fail {};   // a pipeline step failed: r360_last_error() holds the reason

void req_rc(int rc) { if (rc < 0) throw Fail{}; }

float* record(r360_sequence* s, int rep, int pair) {
    return s->job.out + ((size_t)rep * (s->job.p1 - s->job.p0) + (pair - s->job.p0)) * REC;
}

void load_frame(r360_sequence* s, r360_frame* f, int i) {
    const int k = i - s->job.p0;
    if (s->job.device_inputs) req_rc(r360_frame_upload_device(f, s->job.bgr[k], s->job.dep[k]));
    else req_rc(r360_frame_upload_async(f, static_cast<const uint8_t*>(s->job.bgr[k]),
                                        static_cast<const uint16_t*>(s->job.dep[k])));
}

void fill(float* rec, const float pose[16], const float info[36], int status, const r360_icp_stats& st) {
    std::memcpy(rec, pose, sizeof(float) * 16);
    std::memcpy(rec + 16, info, sizeof(float) * 36);
    rec[52] = float(status);
    rec[53] = st.sso;
    rec[54] = float(st.error);
}

const float kEye[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};

// The frame positions of pipeline p's piece: frame index, repeat, and whether positions t, t + 1 form a pair.
struct Positions {
    std::vector<int> frame, rep;
    std::vector<char> pair;
};
Positions positions_of(const r360_sequence* s, int p) {
    Positions P;
    for (const auto& g : s->job.piece[p])
        for (int i = g.a; i <= g.b; ++i) {
            P.frame.push_back(i);
            P.rep.push_back(g.rep);
            P.pair.push_back(i < g.b);
        }
    return P;
}

// No dense queue: the pairs one by one on the pipeline's own context, the reference's sequential Register().
void pipeline_plain(r360_sequence* s, int p) {
    r360_ctx* ctx = s->ctx[p];
    auto& hs = s->host_s[p];
    const int wl = s->prm.workload;
    const Positions X = positions_of(s, p);
    const int T = (int)X.frame.size();
    r360_frame* fa = s->ring[p][0];
    r360_frame* fb = s->ring[p][1];
    load_frame(s, fa, X.frame[0]);
    req_rc(r360_frame_build_async(fa, s->flags));
    for (int t = 0; t + 1 < T; ++t) {
        const double t0 = now_s();
        load_frame(s, fb, X.frame[t + 1]);
        const double tu = now_s();
        req_rc(r360_frame_build_async(fb, s->flags));
        const double t1 = now_s();
        hs[5] += tu - t0;
        hs[4] += t1 - tu;
        if (X.pair[t]) {
            float pose[16], info[36] = {0};
            std::memcpy(pose, kEye, sizeof pose);
            r360_icp_stats st{};
            int status = 0;
            if (wl == R360_SEQ_PLANES) {          // configs[1]: RegisterPbMap alone
                const int rc = r360_register_pbmap(ctx, fa, fb, s->prm.max_match_planes, s->prm.mode, pose, info,
                                                   nullptr, 0, nullptr, nullptr, nullptr, nullptr);
                req_rc(rc);
                status = rc == 1 ? 0 : 1;
                hs[0] += t1 - t0; hs[1] += now_s() - t1; hs[3] += 1;
            } else if (wl == R360_SEQ_DENSE) {    // configs[2] / [4]: alignFrames360 from identity
                req_rc(r360_align360_async(ctx, fa, fb, kEye, R360_PHOTO_DEPTH, 0, &s->prm.icp));
                float dense[16];
                req_rc(r360_align360_result(ctx, dense, nullptr, nullptr, &st));
                rig_from_dense(dense, pose);
                hs[0] += t1 - t0; hs[2] += now_s() - t1; hs[3] += 1;
            } else {                              // configs[3]: the Register() alias
                req_rc(r360_register_async(ctx, fa, fb, kEye, &s->prm.icp, s->prm.max_match_planes, s->prm.mode));
                const double t2 = now_s();
                const int rc = r360_register_result(ctx, pose, info, &st);
                req_rc(rc);
                status = rc;
                hs[0] += t1 - t0; hs[1] += t2 - t1; hs[2] += now_s() - t2; hs[3] += 1;
            }
            if (st.illposed) status = 2;
            fill(record(s, X.rep[t], X.frame[t]), pose, info, status, st);
        } else {
            hs[0] += t1 - t0;
        }
        std::swap(fa, fb);
    }
}

void pipeline_queued(r360_sequence* s, int p) {
    r360_ctx* ctx = s->ctx[p];
    auto& hs = s->host_s[p];
    const int wl = s->prm.workload;
    const Positions X = positions_of(s, p);
    const int T = (int)X.frame.size();
    const std::vector<r360_frame*>& fr = s->ring[p];
    const int nbuf = (int)fr.size();
    const int LA = s->prm.lookahead;
    auto buf = [&](int t) { return fr[t % nbuf]; };

    struct Pending { long ticket; int t; r360_icp_stats st; };
    std::deque<Pending> pending;
    auto finish_front = [&]() {
        Pending pd = pending.front();
        pending.pop_front();
        float pose[16], info[36] = {0};
        int status;
        if (wl == R360_SEQ_DENSE) {
            float dense[16];
            req_rc(r360_dense_queue_collect(s->q, pd.ticket, dense, nullptr, nullptr, &pd.st));
            rig_from_dense(dense, pose);
            status = 0;
        } else {
            const int rc = r360_register_collect(s->q, pd.ticket, pose, info, &pd.st);
            req_rc(rc);
            status = rc;
        }
        if (pd.st.illposed) status = 2;
        fill(record(s, X.rep[pd.t], X.frame[pd.t]), pose, info, status, pd.st);
    };
    auto load = [&](int t) {
        const double u0 = now_s();
        load_frame(s, buf(t), X.frame[t]);
        hs[5] += now_s() - u0;
    };
    auto build = [&](int t) {
        const double b0 = now_s();
        req_rc(r360_frame_build_async(buf(t), s->flags));
        hs[4] += now_s() - b0;
    };

    const int last = T - 1;
    // A failed step leaves no ticket behind: every pending job is collected (its result, or error, dropped) before
    // the failure propagates, so the dense queue holds no job that reads this pipeline's frames once the run returns
    // (a later run refills them, r360_sequence_destroy frees them) and none of its job entries leak.
    try {
        for (int t = 0; t < std::min(LA, last + 1); ++t) {   // positions 0 .. LA-1 built, position LA uploaded
            load(t);
            build(t);
        }
        if (LA <= last) load(LA);
        const int depth = nbuf - LA - 2;
        for (int t = 0; t < last; ++t) {
            const double t0 = now_s();
            // position t + LA + 1 refills the buffer of position u = t + LA + 1 - nbuf: collect the pairs that used it
            while (!pending.empty() && pending.front().t <= t + LA + 1 - nbuf) finish_front();
            hs[6] += now_s() - t0;
            r360_frame* cur = buf(t);
            r360_frame* nxt = buf(t + 1);
            if (t + LA <= last) build(t + LA);                  // its upload was issued one iteration earlier
            if (t + LA + 1 <= last) load(t + LA + 1);
            const double t1 = now_s();
            if (!X.pair[t]) {                                   // the last frame of a segment: no pair
                hs[0] += t1 - t0;
                continue;
            }
            long ticket = 0;
            if (wl == R360_SEQ_DENSE)
                req_rc(r360_dense_queue_submit(s->q, cur, nxt, kEye, R360_PHOTO_DEPTH, &s->prm.icp, &ticket));
            else
                req_rc(r360_register_submit(ctx, s->q, cur, nxt, kEye, &s->prm.icp, s->prm.max_match_planes, s->prm.mode,
                                            &ticket));
            const double t2 = now_s();
            pending.push_back(Pending{ticket, t, r360_icp_stats{}});
            if ((int)pending.size() > depth) finish_front();
            hs[0] += t1 - t0; hs[1] += t2 - t1; hs[2] += now_s() - t2; hs[3] += 1;
        }
        const double t2 = now_s();
        while (!pending.empty()) finish_front();
        hs[2] += now_s() - t2;
    } catch (...) {
        const std::string why = r360_last_error();
        for (const Pending& pd : pending) {
            float pose[16], info[36];
            r360_icp_stats st{};
            if (wl == R360_SEQ_DENSE) (void)r360_dense_queue_collect(s->q, pd.ticket, pose, nullptr, nullptr, &st);
            else (void)r360_register_collect(s->q, pd.ticket, pose, info, &st);
        }
        pending.clear();
        r360_set_error("%s", why.c_str());   // the first failure, not a drained job's
        throw;
    }
}

void worker(r360_sequence* s, int p) {
    (void)hipSetDevice(s->device);
    {
        std::lock_guard<std::mutex> lk(s->m);
        s->tid[p] = (long)syscall(SYS_gettid);
    }
    s->cv_done.notify_all();
    long seen = 0;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(s->m);
            s->cv_go.wait(lk, [&] { return s->quit || s->gen != seen; });
            if (s->quit) return;
            seen = s->gen;
        }
        int rc = 0;
        std::string err;
        if (p < (int)s->job.piece.size() && !s->job.piece[p].empty()) {
            // experiment builds: start pipeline p p x R360_SEQ_STAGGER_US later
            static const int stagger_us = R360_KNOB("R360_SEQ_STAGGER_US", 0);
            if (stagger_us) std::this_thread::sleep_for(std::chrono::microseconds((long)p * stagger_us));
            try {
                if (s->q) pipeline_queued(s, p);
                else pipeline_plain(s, p);
            } catch (const Fail&) {
                rc = -1;
                err = r360_last_error();
            } catch (const std::exception& e) {
                rc = -1;
                err = std::string("pipeline: ") + e.what();
            }
        }
        std::lock_guard<std::mutex> lk(s->m);
        s->rc[p] = rc;
        s->err[p] = err;
        ++s->done;
        s->cv_done.notify_all();
    }
}

}  // namespace

extern "C" void r360_sequence_default_params(r360_sequence_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->rows = 480; p->cols = 640;
    p->pipelines = 10;
    p->queue = 16;
    p->depth = 3;
    p->lookahead = 1;
    p->plane_batch = R360_PLANE_BATCH;
    p->workload = R360_SEQ_FULL;
    p->max_match_planes = 25;
    p->mode = R360_PLANAR_3DoF;
    r360_icp_default_params(&p->icp);
    p->icp.n_pyr = 5;                              // OdometryRGBD360.cpp:92-95
    p->icp.std_dev_photo = 3.0f / 255;
    p->icp.fixed_iters_level0 = 20;               // timing mode
}

extern "C" void r360_sequence_destroy(r360_sequence* s);
int plane_queue_reserve(r360_plane_queue* q, const PlaneGeom& G);   // plane_queue.cpp
int dense_queue_reserve(r360_dense_queue* q, long n_pixels);          // dense_queue.cpp

extern "C" int r360_sequence_create(int device, const r360_sequence_params* prm, const char* extrinsics_dir,
                                    r360_sequence** out) {
    CHECK_ARG(prm && out, "null arg");
    CHECK_ARG(prm->pipelines >= 1 && prm->pipelines <= 64, "pipelines must be 1..64");
    CHECK_ARG(prm->rows > 0 && prm->cols > 0, "rows / cols");
    CHECK_ARG(prm->workload >= R360_SEQ_FULL && prm->workload <= R360_SEQ_DENSE, "workload");
    CHECK_ARG(prm->queue >= 0 && prm->queue <= R360_MAX_BATCH, "queue must be 0..R360_MAX_BATCH_ALIGN");
    CHECK_ARG(prm->plane_batch >= 0 && prm->plane_batch <= R360_PLANE_BATCH, "plane_batch must be 0..8");
    if (bind_device(device)) return -1;
    std::unique_ptr<r360_sequence> s(new r360_sequence);
    s->device = device;
    s->prm = *prm;
    if (s->prm.workload == R360_SEQ_PLANES) s->prm.queue = 0;   // no dense stage
    s->prm.depth = std::max(1, s->prm.depth);
    s->prm.lookahead = std::max(1, s->prm.lookahead);
    s->P = prm->pipelines;
    // configs[1] needs the planes only, configs[2] / [4] the sphere pyramid only
    s->flags = s->prm.workload == R360_SEQ_PLANES ? (R360_BUILD_UNDISTORT | R360_BUILD_PLANES)
             : s->prm.workload == R360_SEQ_DENSE ? (R360_BUILD_UNDISTORT | R360_BUILD_SPHERE | R360_BUILD_PYRAMID)
             : (R360_BUILD_UNDISTORT | R360_BUILD_SPHERE | R360_BUILD_PYRAMID | R360_BUILD_PLANES);
    auto fail = [&]() {
        r360_sequence_destroy(s.release());
        return -1;
    };
    if (s->prm.queue > 0 && r360_dense_queue_create(device, s->prm.queue, &s->q)) return fail();
    const bool queued = s->q != nullptr;
    if (s->prm.workload != R360_SEQ_DENSE && s->prm.plane_batch > 0 &&
        plane_queue_create(device, s->prm.plane_batch, &s->pq))
        return fail();
    const int nbuf = queued ? s->prm.depth + s->prm.lookahead + 2 : 2;
    for (int p = 0; p < s->P; ++p) {
        r360_ctx* c = nullptr;
        if (r360_ctx_create(device, &c)) return fail();
        s->ctx.push_back(c);
        c->plane_q = s->pq;
        // a single pipeline waits for each new frame's PbMap (the sequential caller): its thread helps assemble it;
        // several pipelines leave it to the assembly pool (spinning waits would take the host cores it needs)
        if (r360_ctx_latency_mode(c, s->P == 1)) return fail();
        // experiment builds: R360_SEQ_SHARE=k puts the first k pipelines' work on the dense queue's stream
        static const int share = R360_KNOB("R360_SEQ_SHARE", 0);
        if (queued && p < share) {
            R360_HIP(hipStreamSynchronize(c->stream));
            R360_HIP(hipStreamDestroy(c->stream));
            c->stream = r360_dense_queue_ctx(s->q)->stream;
            c->stream_borrowed = true;
        }
        r360_calib* k = nullptr;
        if (r360_calib_create(c, prm->rows, prm->cols, &k)) return fail();
        s->cal.push_back(k);
        if (r360_calib_load_extrinsics(k, extrinsics_dir)) return fail();
        s->ring.emplace_back();
        for (int j = 0; j < nbuf; ++j) {
            r360_frame* f = nullptr;
            if (r360_frame_create(c, k, &f)) return fail();
            s->ring.back().push_back(f);
            // queued alignments are batched (PF 6 / PF 8 stream the images): no compacted source points
            if (s->q) f->compact_all = false;
            // the pyramid the alignments use (setNumPyr): deeper levels would be built for nothing
            if (s->prm.workload != R360_SEQ_PLANES && s->prm.icp.n_pyr < f->n_levels &&
                r360_frame_set_levels(f, s->prm.icp.n_pyr))
                return fail();
        }
    }
    // every buffer the runs size on first use, sized now: a short run (one rank's shard: a few pairs per pipeline
    // and step) would otherwise allocate inside its timed steps, and hipMalloc synchronises the device
    {
        r360_frame* f0 = s->ring[0][0];
        const long npx = (long)f0->lv[0].rows * f0->lv[0].cols;
        if (s->flags & R360_BUILD_PLANES) {
            for (auto& r : s->ring)
                for (r360_frame* f : r)
                    if (plane_bufs_alloc(f)) return fail();
            const PlaneGeom G = plane_geom(f0);
            if (s->pq) {
                if (plane_queue_reserve(s->pq, G)) return fail();
            } else {
                long cells, entries, groups;
                vox_scratch_need(G, &cells, &entries, &groups);
                for (r360_ctx* c : s->ctx)
                    if (ctx_vhash_reserve(c, cells, entries, groups)) return fail();
            }
        }
        if (s->prm.workload != R360_SEQ_PLANES) {
            if (s->q) {
                if (dense_queue_reserve(s->q, npx)) return fail();
            } else {
                for (r360_ctx* c : s->ctx)
                    if (ensure_defer(c, npx)) return fail();
            }
        }
        R360_HIP(hipDeviceSynchronize());
    }
    s->tid.assign(s->P, 0);
    s->rc.assign(s->P, 0);
    s->err.assign(s->P, std::string());
    s->host_s.assign(s->P, std::array<double, 8>{});
    for (int p = 0; p < s->P; ++p) s->th.emplace_back(worker, s.get(), p);
    {   // the threads' ids (host CPU accounting of the callers)
        std::unique_lock<std::mutex> lk(s->m);
        s->cv_done.wait(lk, [&] {
            for (long t : s->tid) if (!t) return false;
            return true;
        });
    }
    *out = s.release();
    return 0;
}

extern "C" void r360_sequence_destroy(r360_sequence* s) {
    if (!s) return;
    {
        std::lock_guard<std::mutex> lk(s->m);
        s->quit = true;
    }
    s->cv_go.notify_all();
    for (auto& t : s->th) t.join();
    // the queues first: their dispatchers drain what is still queued, which reads the ring frames
    if (s->q) r360_dense_queue_destroy(s->q);
    if (s->pq) plane_queue_destroy(s->pq);
    for (auto& r : s->ring)
        for (r360_frame* f : r) {
            planes_join(f);
            r360_frame_destroy(f);
        }
    for (r360_calib* k : s->cal) r360_calib_destroy(k);
    for (r360_ctx* c : s->ctx) r360_ctx_destroy(c);
    delete s;
}

extern "C" int r360_sequence_run(r360_sequence* s, int p0, int p1, const void* const* bgr, const void* const* depth,
                                 int device_inputs, int repeats, const int* runs, int n_runs, float* records) {
    CHECK_ARG(s && bgr && depth && records, "null arg");
    CHECK_ARG(p1 > p0 && repeats >= 1, "empty run");
    if (bind_device(s->device)) return -1;
    const int n = p1 - p0;
    std::vector<std::vector<r360_sequence::Seg>> piece(s->P);
    if (runs && n_runs > 0) {   // every repeat split the same way: pipeline k takes run k of each repeat
        CHECK_ARG(n_runs <= s->P, "more runs than pipelines");
        int at = p0;
        for (int k = 0; k < n_runs; ++k) {
            CHECK_ARG(runs[2 * k] == at && runs[2 * k + 1] > runs[2 * k], "runs must tile [p0, p1) in order");
            for (int r = 0; r < repeats; ++r) piece[k].push_back({r, runs[2 * k], runs[2 * k + 1]});
            at = runs[2 * k + 1];
        }
        CHECK_ARG(at == p1, "runs must tile [p0, p1)");
    } else {   // the repeats x n pair registrations as one stream, cut into P near-equal contiguous pieces
        const long total = (long)repeats * n;
        const int parts = (int)std::min<long>(s->P, total);
        long at = 0;
        for (int k = 0; k < parts; ++k) {
            const long e = at + total / parts + (k < total % parts ? 1 : 0);
            for (long u = at; u < e;) {            // u = r * n + (i - p0)
                const int r = (int)(u / n), i = (int)(u % n);
                const int b = (int)std::min<long>(n, i + (e - u));
                piece[k].push_back({r, p0 + i, p0 + b});
                u += b - i;
            }
            at = e;
        }
    }
    s->job.p0 = p0; s->job.p1 = p1; s->job.repeats = repeats; s->job.device_inputs = device_inputs;
    s->job.piece = std::move(piece);
    s->job.bgr = bgr; s->job.dep = depth; s->job.out = records;
    {
        std::lock_guard<std::mutex> lk(s->m);
        s->done = 0;
        ++s->gen;
    }
    s->cv_go.notify_all();
    {
        std::unique_lock<std::mutex> lk(s->m);
        s->cv_done.wait(lk, [&] { return s->done == s->P; });
    }
    for (r360_ctx* c : s->ctx) if (r360_ctx_sync(c)) return -1;
    for (int p = 0; p < s->P; ++p)
        if (s->rc[p]) {
            r360_set_error("%s", s->err[p].c_str());
            return -1;
        }
    return 0;
}

extern "C" int r360_sequence_info(r360_sequence* s, int* pipelines, r360_dense_queue** queue) {
    CHECK_ARG(s, "null sequence");
    if (pipelines) *pipelines = s->P;
    if (queue) *queue = s->q;
    return 0;
}

extern "C" int r360_sequence_plane_stats(r360_sequence* s, long* batches, long* frames, int* max_batch_seen,
                                         r360_ctx** ctx) {
    CHECK_ARG(s, "null sequence");
    if (ctx) *ctx = plane_queue_ctx(s->pq);
    if (!s->pq) {
        if (batches) *batches = 0;
        if (frames) *frames = 0;
        if (max_batch_seen) *max_batch_seen = 0;
        return 0;
    }
    return plane_queue_stats(s->pq, batches, frames, max_batch_seen);
}

extern "C" int r360_sequence_pipeline(r360_sequence* s, int p, r360_ctx** ctx, r360_calib** calib, r360_frame** frames,
                                      int cap, int* n_frames, long* thread_id) {
    CHECK_ARG(s && p >= 0 && p < s->P, "pipeline out of range");
    if (ctx) *ctx = s->ctx[p];
    if (calib) *calib = s->cal[p];
    const int n = (int)s->ring[p].size();
    if (n_frames) *n_frames = n;
    for (int j = 0; j < n && j < cap && frames; ++j) frames[j] = s->ring[p][j];
    if (thread_id) {
        std::lock_guard<std::mutex> lk(s->m);
        *thread_id = s->tid[p];
    }
    return 0;
}

extern "C" int r360_sequence_host_times(r360_sequence* s, double* out, int reset) {
    CHECK_ARG(s, "null sequence");
    std::lock_guard<std::mutex> lk(s->m);
    for (int p = 0; p < s->P; ++p)
        for (int k = 0; k < 8; ++k) {
            if (out) out[8 * p + k] = s->host_s[p][k];
            if (reset) s->host_s[p][k] = 0;
        }
    return 0;
}
