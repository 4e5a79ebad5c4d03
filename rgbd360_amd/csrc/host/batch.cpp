// Batched pair registrations: SphereGraphSLAM's tracking loop and LoopClosure360's
// candidate checks issue many independent RegisterPbMap / alignFrames360 calls per frame
// (SLAM/SphereGraphSLAM.cpp:169-231, include/LoopClosure360.h:280-366).  The reference runs them one
// after another on one RegisterRGBD360 / RegisterPhotoICP object.  Here a batch owns `lanes` worker
// contexts (each with its own HIP stream, device GN state and matcher scratch) and one host thread per
// lane (persistent workers), so the host interpretation-tree searches of different pairs overlap each other and the dense
// refinements of different pairs run side by side on the GPU.  Every job is the unchanged single-pair
// code path (r360_register_pbmap, r360_align360_async/_result), so batched results are identical to
// sequential ones.
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../r360_internal.h"


struct r360_batch {
    int device = 0;
    std::vector<r360_ctx*> lane;
    std::vector<hipEvent_t> dep;   // one "frame built" event per distinct frame of a call (grown on demand)
    // persistent workers for lanes 1..L-1 (the calling thread drives lane 0): a call publishes `task` under a
    // new generation number and waits until every worker has run it
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable go, done;
    unsigned long gen = 0;
    int busy = 0;
    bool stop = false;
    std::function<void(int)> task;
    std::recursive_mutex call;   // one call at a time (r360_track_frame re-enters r360_batch_register): a second caller waits instead of overwriting task / lane state

    void worker(int l) {
        hipSetDevice(device);
        unsigned long seen = 0;
        for (;;) {
            std::function<void(int)> t;
            {
                std::unique_lock<std::mutex> lk(m);
                go.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
                t = task;
            }
            t(l);
            std::lock_guard<std::mutex> lk(m);
            if (--busy == 0) done.notify_all();
        }
    }
    void run(const std::function<void(int)>& fn) {
        {
            std::lock_guard<std::mutex> lk(m);
            task = fn;
            busy = int(th.size());
            ++gen;
        }
        go.notify_all();
        fn(0);
        std::unique_lock<std::mutex> lk(m);
        done.wait(lk, [&] { return busy == 0; });
    }
};

extern "C" int r360_batch_create(int device, int lanes, r360_batch** out) {
    CHECK_ARG(out, "null out");
    CHECK_ARG(lanes >= 1 && lanes <= 64, "lanes must be 1..64");
    r360_batch* b = new r360_batch;
    b->device = device;
    for (int i = 0; i < lanes; ++i) {
        r360_ctx* c = nullptr;
        if (int rc = r360_ctx_create(device, &c)) { r360_batch_destroy(b); return rc; }
        b->lane.push_back(c);
    }
    for (int l = 1; l < lanes; ++l) b->th.emplace_back(&r360_batch::worker, b, l);
    *out = b;
    return 0;
}

extern "C" void r360_batch_destroy(r360_batch* b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> lk(b->m);
        b->stop = true;
    }
    b->go.notify_all();
    for (auto& t : b->th) t.join();
    for (auto c : b->lane) r360_ctx_destroy(c);
    hipSetDevice(b->device);
    for (auto e : b->dep) hipEventDestroy(e);
    delete b;
}

extern "C" int r360_batch_lanes(const r360_batch* b) { return b ? int(b->lane.size()) : 0; }

extern "C" int r360_batch_set_match_params(r360_batch* b, const r360_match_params* m) {
    CHECK_ARG(b && m, "null arg");
    std::lock_guard<std::recursive_mutex> serial(b->call);
    for (auto c : b->lane)
        if (int rc = r360_ctx_set_match_params(c, m)) return rc;
    return 0;
}

namespace {

void identity16(float* m) {
    for (int i = 0; i < 16; ++i) m[i] = (i % 5 == 0) ? 1.f : 0.f;
}

struct FrameDeps {
    std::unordered_map<r360_frame*, hipEvent_t> ev;
};

// Host-side readiness of every distinct frame, on the calling thread (the PbMap assembly join of a frame
// must not race between lanes), and one event per frame marking the end of its build work on its own
// ctx's stream, for the lanes' streams to wait on.
int prepare_frames(r360_batch* b, const std::vector<r360_frame*>& frames, bool need_planes, FrameDeps& D) {
    size_t k = 0;
    for (r360_frame* f : frames) {
        CHECK_ARG(f && f->ctx, "null frame");
        CHECK_ARG(f->ctx->device == b->device, "frame belongs to another device");
        if (D.ev.count(f)) continue;
        if (need_planes) {
            CHECK_ARG(f->built & R360_BUILD_PLANES, "frame planes not built (R360_BUILD_PLANES)");
            if (int rc = planes_finish(f)) return rc;
        }
        if (k == b->dep.size()) {
            hipEvent_t e;
            R360_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            b->dep.push_back(e);
        }
        R360_HIP(hipEventRecord(b->dep[k], f->ctx->stream));
        D.ev[f] = b->dep[k++];
    }
    return 0;
}

int wait_frames(r360_ctx* lane, const FrameDeps& D, r360_frame* a, r360_frame* c) {
    for (r360_frame* f : {a, c})
        if (f->ctx != lane) R360_HIP(hipStreamWaitEvent(lane->stream, D.ev.at(f), 0));
    return 0;
}

// One job on one lane: RegisterPbMap (RegisterRGBD360.h:276-337), then the dense stage the job asks for.
int run_job(r360_ctx* lane, const FrameDeps& D, const r360_pair_job& j, size_t max_match_planes, int mode,
            int min_matches, float min_area, const r360_icp_params* p, r360_pair_result& r) {
    memset(&r, 0, sizeof r);
    identity16(r.pbmap_pose);
    identity16(r.pose);
    r.dense_rc = -1;
    if (int rc = wait_frames(lane, D, j.ref, j.trg)) return rc;
    const int good = r360_register_pbmap(lane, j.ref, j.trg, max_match_planes, mode, r.pbmap_pose, r.pbmap_info,
                                         nullptr, 0, &r.n_match, &r.area_matched, &r.area_src, &r.area_trg);
    if (good < 0) return good;
    r.good = good;
    if (good == 1 && r.area_src > 0.f) r.sso_pbmap = r.area_matched / r.area_src;
    bool dense = false;
    const float* start = r.pbmap_pose;
    if (j.dense == R360_JOB_GATED) {
        dense = good == 1 && r.n_match > min_matches && r.area_matched > min_area;
    } else if (j.dense == R360_JOB_ALWAYS) {
        dense = true;
        if (good != 1) start = j.guess;
    }
    if (!dense) return 0;
    float Ro[16], Ri[16], t[16], init[16];
    r360_rot_offset(Ro, Ri);
    r360_mul4(Ro, start, t);
    r360_mul4(t, Ri, init);                                  // rotOffset * relativePose * rotOffset^-1
    r360_frame* trg = j.ref_is_source ? j.trg : j.ref;       // setTargetFrame
    r360_frame* src = j.ref_is_source ? j.ref : j.trg;       // setSourceFrame
    if (int rc = r360_align360_async(lane, trg, src, init, R360_PHOTO_DEPTH, 0, p)) return rc;
    float opt[16];
    const int rc = r360_align360_result(lane, opt, r.hessian, nullptr, &r.stats);
    if (rc < 0) return rc;
    r.dense_rc = rc;
    r360_mul4(Ri, opt, t);
    r360_mul4(t, Ro, r.pose);                                // rotOffset^-1 * getOptimalPose() * rotOffset
    return 0;
}

}  // namespace

extern "C" int r360_batch_register(r360_batch* b, const r360_pair_job* jobs, int n, size_t max_match_planes,
                                   int mode, int min_matches, float min_area, const r360_icp_params* p,
                                   r360_pair_result* out) {
    CHECK_ARG(b && (n == 0 || (jobs && out)), "null arg");
    CHECK_ARG(n >= 0, "negative job count");
    std::lock_guard<std::recursive_mutex> serial(b->call);
    CHECK_ARG(mode >= 0 && mode <= 3, "registrationType must be 0..3");
    bool any_dense = false;
    std::vector<r360_frame*> frames;
    for (int i = 0; i < n; ++i) {
        CHECK_ARG(jobs[i].dense >= R360_JOB_PBMAP_ONLY && jobs[i].dense <= R360_JOB_ALWAYS, "invalid job dense mode");
        any_dense |= jobs[i].dense != R360_JOB_PBMAP_ONLY;
        frames.push_back(jobs[i].ref);
        frames.push_back(jobs[i].trg);
    }
    CHECK_ARG(!any_dense || p, "dense jobs need ICP parameters");
    if (n == 0) return 0;
    FrameDeps D;
    if (int rc = prepare_frames(b, frames, true, D)) return rc;

    std::atomic<int> next{0};
    std::vector<int> rcs(n, 0);
    std::vector<std::string> errs(n);
    b->run([&](int l) {
        for (int i = next++; i < n; i = next++) {
            rcs[i] = run_job(b->lane[l], D, jobs[i], max_match_planes, mode, min_matches, min_area, p, out[i]);
            if (rcs[i] < 0) errs[i] = r360_last_error();
        }
    });
    for (int i = 0; i < n; ++i)
        if (rcs[i] < 0) {
            r360_set_error("job %d: %s", i, errs[i].c_str());
            return rcs[i];
        }
    return 0;
}

extern "C" int r360_track_frame(r360_batch* b, r360_frame* const* kfs, int n_kf, r360_frame* frame, int num_check,
                                int no_assoc_threshold, size_t max_match_planes, int mode, int* chosen,
                                r360_pair_result* result, r360_pair_result* cand) {
    CHECK_ARG(b && frame && chosen && (n_kf == 0 || kfs), "null arg");
    CHECK_ARG(n_kf >= 0 && num_check >= 0 && no_assoc_threshold >= 0, "negative count");
    std::lock_guard<std::recursive_mutex> serial(b->call);
    // while(compareLocalIdx >= 0 && compareLocalIdx >= newLocalFrameID - numCheckRegistration &&
    //       noAssoc < noAssoc_threshold): every failed candidate increments noAssoc, so at most
    // min(n_kf, num_check, no_assoc_threshold) candidates are tried, newest first
    const int m = std::min(n_kf, std::min(num_check, no_assoc_threshold));
    *chosen = -1;
    if (m == 0) return 0;
    std::vector<r360_pair_job> jobs(m);
    for (int c = 0; c < m; ++c) {
        r360_pair_job& j = jobs[c];
        memset(&j, 0, sizeof j);
        j.ref = kfs[n_kf - 1 - c];
        j.trg = frame;
        j.dense = R360_JOB_PBMAP_ONLY;
        identity16(j.guess);
    }
    std::vector<r360_pair_result> res(m);
    if (int rc = r360_batch_register(b, jobs.data(), m, max_match_planes, mode, 0, 0.f, nullptr, res.data()))
        return rc;
    for (int c = 0; c < m; ++c)
        if (res[c].good == 1) {                  // "break; // Stop the loop when there is a valid registration"
            *chosen = n_kf - 1 - c;
            if (result) *result = res[c];
            break;
        }
    if (cand) memcpy(cand, res.data(), sizeof(r360_pair_result) * m);
    return 0;
}
