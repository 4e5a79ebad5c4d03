"""OdometryRGBD360 over a Frame360 sequence, sharded by pair (BASELINE config 4).

The reference's loop (Registration/OdometryRGBD360.cpp:141-257) walks a sequence, registers each new
Frame360 against the previous one (RegisterPbMap, then alignFrames360) and composes the trajectory with
``currentPose = currentPose * rigidTransf`` (:257).  Registering pair (i, i+1) needs only frames i and
i+1, so the 255 pairs of a 256-frame sequence are split into contiguous shards, one per rank (one
process per GPU), and each rank's shard into contiguous runs, one per pipeline (one ``r360_ctx`` =
host thread + HIP stream).  A pipeline builds the first frame of its run (the halo frame, also built by
the previous run) and then, per pair, uploads and builds the new frame and registers it with the
``Register()`` alias (PbMap -> rotOffset conjugation -> alignFrames360, OdometryKeyFrame360.cpp:205-254).
Every pair is registered exactly once; rank 0 gathers the per-pair records and forms the prefix product.

Deviation, by construction of the sharding: the reference's ``dist < 0.4`` keyframe skip (:230-238)
makes pair i depend on earlier results (the reference frame only advances after a far-enough frame), so
a sharded run registers consecutive pairs.  ``apps/OdometryRGBD360`` keeps the skip for sequential runs.
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor

import time

import numpy as np

from . import (BUILD_PLANES, BUILD_PYRAMID, BUILD_SPHERE, BUILD_UNDISTORT, PHOTO_DEPTH, PLANAR_3DoF, Calib360,
               Context, DenseQueue, Frame360, IcpParams, IcpStats, EXTRINSICS_DIR, C, _fptr, lib)

SEQ_FRAMES = 256
# one pair record: pose (16, column-major, rig frame of the pair's first frame), the PbMap information
# matrix (36), status (0: PbMap stage good, 1: PbMap failed and the dense stage started from the guess,
# 2: alignFrames360 ill-posed), SSO, the accepted level-0 error
REC = 56

# rotOffset of OdometryRGBD360.cpp:136-139 (the sphere's frame vs the rig's), float angle, double PI
_A = float(np.float32(157.5)) * 3.14159265359 / 180
ROT_OFFSET = np.eye(4)
ROT_OFFSET[1, 1] = ROT_OFFSET[2, 2] = np.float32(np.cos(_A))
ROT_OFFSET[1, 2], ROT_OFFSET[2, 1] = np.float32(np.sin(_A)), -np.float32(np.sin(_A))
ROT_OFFSET_INV = ROT_OFFSET.T.copy()
R_POSE, R_INFO, R_STATUS, R_SSO, R_ERR = 0, 16, 52, 53, 54


def split_range(a: int, b: int, parts: int) -> list[tuple[int, int]]:
    """[a, b) in `parts` contiguous pieces whose sizes differ by at most one (empty pieces dropped)."""
    n = b - a
    parts = max(1, min(parts, n)) if n > 0 else 1
    base, extra = divmod(n, parts)
    out, s = [], a
    for k in range(parts):
        e = s + base + (1 if k < extra else 0)
        if e > s:
            out.append((s, e))
        s = e
    return out


def shard_pairs(rank: int, world: int, n_frames: int = SEQ_FRAMES) -> tuple[int, int]:
    """Pairs [p0, p1) of rank `rank`: pair i registers frames (i, i+1); the n_frames-1 pairs are split
    contiguously over the ranks.  The rank needs frames p0..p1."""
    n = n_frames - 1
    base, extra = divmod(n, world)
    p0 = rank * base + min(rank, extra)
    return p0, p0 + base + (1 if rank < extra else 0)


def pipelines_for(n_pairs: int, streams: int, min_run: int) -> int:
    """Pipelines for a shard: at most `streams`, each with a run of at least `min_run` pairs (every run
    rebuilds its halo frame, so short runs cost extra frame builds)."""
    return max(1, min(streams, n_pairs // max(1, min_run)))


def compose(records: np.ndarray) -> np.ndarray:
    """Trajectory of the sequence: T[0] = I, T[k+1] = T[k] * pose_k (OdometryRGBD360.cpp:257), in float64."""
    n = records.shape[0]
    T = np.zeros((n + 1, 4, 4))
    T[0] = np.eye(4)
    for k in range(n):
        T[k + 1] = T[k] @ records[k, R_POSE:R_POSE + 16].reshape(4, 4).T.astype(np.float64)
    return T


def trajectory_error(T: np.ndarray, gt: np.ndarray) -> dict:
    """Per-frame error of a composed trajectory against ground-truth rig poses gt[k] (composed from gt[0])."""
    g0 = np.linalg.inv(gt[0])
    rot, trans = [], []
    for k in range(T.shape[0]):
        G = g0 @ gt[k]
        D = np.linalg.inv(G) @ T[k]
        rot.append(float(np.degrees(np.arccos(np.clip((np.trace(D[:3, :3]) - 1) / 2, -1, 1)))))
        trans.append(float(np.linalg.norm(T[k][:3, 3] - G[:3, 3])))
    path = float(sum(np.linalg.norm(gt[k + 1][:3, 3] - gt[k][:3, 3]) for k in range(len(gt) - 1)))
    return {"frames": int(T.shape[0]), "max_rot_err_deg": max(rot), "max_trans_err_m": max(trans),
            "final_rot_err_deg": rot[-1], "final_trans_err_m": trans[-1], "path_length_m": path}


EDGE_WAIT_S = 120.0   # a shared edge frame not built / released within this time: the neighbour pipeline is stuck


class SequenceRunner:
    """P pipelines on one GPU, each an r360_ctx (HIP stream + device GN state) driven by its own host thread
    (ctypes drops the GIL inside the library), each with two Frame360 buffers used in turn.

    queue > 0: the pipelines' alignFrames360 calls go to one dense queue (r360_dense_queue, batches of up to
    `queue` pairs per launch on the queue's stream) and each pipeline keeps one alignment in flight while it
    builds and PbMap-registers the next frame (three Frame360 buffers in turn).  Every record is identical to
    the unqueued run's (a batched alignment equals the single-pair one bit for bit)."""

    def __init__(self, device: int, rows: int, cols: int, pipelines: int, params: IcpParams,
                 planes: bool = True, max_match_planes: int = 25, mode: int = PLANAR_3DoF, dense_only: bool = False,
                 queue: int = 0, planes_only: bool = False, depth: int = 1, lookahead: int = 1,
                 share_edges: bool = True):
        self.P = pipelines
        self.lookahead = max(1, lookahead)   # queued mode: frames whose build is enqueued ahead of the pair in hand
        self.dense_only = dense_only
        self.planes_only = planes_only
        if planes_only:
            queue = 0
        self.queue = DenseQueue(device, queue) if queue > 0 else None
        self.depth = max(1, depth)   # queued mode: alignments in flight per pipeline
        self.params = params
        self.max_match_planes, self.mode = max_match_planes, mode
        self.flags = BUILD_UNDISTORT | BUILD_SPHERE | BUILD_PYRAMID | (BUILD_PLANES if planes else 0)
        self.ctxs = [Context(device) for _ in range(pipelines)]
        self.cals, self.frames = [], []
        for c in self.ctxs:
            cal = Calib360(c, rows, cols)
            cal.loadExtrinsicCalibration(EXTRINSICS_DIR)
            self.cals.append(cal)
            # queued: depth alignments in flight, the pair being registered, the frames built ahead and the next
            # frame's prefetched upload
            self.frames.append([Frame360(cal) for _ in range(self.depth + self.lookahead + 2 if self.queue else 2)])
        # queued mode: the frame where pipeline p's run starts is also where pipeline p-1's run ends; pipeline p
        # builds it (in a buffer of its own, outside its ring) and pipeline p-1 registers its last pair against
        # it, so contiguous runs cost no halo frame builds (share_edges=False: each pipeline builds both)
        self.share_edges = bool(self.queue) and share_edges
        self.edge_frames = [Frame360(cal) for cal in self.cals] if self.share_edges else None
        self.edges = None
        self.stats = [IcpStats() for _ in range(pipelines)]
        # host-side time per pipeline: [load + build enqueue, PbMap stage (register_async), dense wait, pairs]
        self.host_s = np.zeros((pipelines, 4))
        self.pool = ThreadPoolExecutor(max_workers=pipelines)
        self.native_ids = set()   # OS thread ids of the pipeline threads (host CPU accounting)
        self.eye = np.eye(4, dtype=np.float32).reshape(16)

    def _pipeline(self, p: int, run: tuple[int, int], frames_of, out: np.ndarray, p0: int, device_inputs: bool):
        """Pipeline p registers pairs run[0]..run[1]-1; out[i - p0] = the record of pair i.  Frame i's raw
        images come from frames_of(i): host arrays (uploaded over PCIe) or, with device_inputs, device
        pointers of images already resident in HBM (copied device to device)."""
        L = lib()
        ctx = self.ctxs[p]
        fa, fb = self.frames[p]
        a, b = run

        def load(f, i):
            if device_inputs:
                f.upload_device(*frames_of(i))
            else:
                f.upload_async(*frames_of(i))
        hs = self.host_s[p]
        load(fa, a)
        fa.build(self.flags, sync=False)
        for i in range(a, b):
            t0 = time.perf_counter()
            load(fb, i + 1)
            fb.build(self.flags, sync=False)
            t1 = time.perf_counter()
            rec = out[i - p0]
            pose, info = np.zeros(16, np.float32), np.zeros(36, np.float32)
            if self.planes_only:   # configs[1]: the PbMap stage alone (RegisterPbMap), no alignFrames360
                rc = L.r360_register_pbmap(ctx.h, fa.h, fb.h, self.max_match_planes, self.mode, _fptr(pose),
                                           _fptr(info), None, 0, None, None, None, None)
                if rc < 0:
                    raise RuntimeError(f"r360_register_pbmap: {L.r360_last_error()}")
                rc = 0 if rc == 1 else 1
                hs += (t1 - t0, time.perf_counter() - t1, 0, 1)
            elif self.dense_only:   # alignFrames360 from identity (configs 3 / 5), pose conjugated back to the rig
                rc = L.r360_align360_async(ctx.h, fa.h, fb.h, _fptr(self.eye), PHOTO_DEPTH, 0, C.byref(self.params))
                if rc != 0:
                    raise RuntimeError(f"r360_align360_async: {L.r360_last_error()}")
                dense = np.zeros(16, np.float32)
                rc = L.r360_align360_result(ctx.h, _fptr(dense), None, None, C.byref(self.stats[p]))
                if rc < 0:
                    raise RuntimeError(f"r360_align360_result: {L.r360_last_error()}")
                pose = (ROT_OFFSET_INV @ dense.reshape(4, 4).T.astype(np.float64) @ ROT_OFFSET).T.reshape(16)
                rc = 0
            else:
                rc = L.r360_register_async(ctx.h, fa.h, fb.h, _fptr(self.eye), C.byref(self.params),
                                           self.max_match_planes, self.mode)
                if rc != 0:
                    raise RuntimeError(f"r360_register_async: {L.r360_last_error()}")
                t2 = time.perf_counter()
                rc = L.r360_register_result(ctx.h, _fptr(pose), _fptr(info), C.byref(self.stats[p]))
                if rc < 0:
                    raise RuntimeError(f"r360_register_result: {L.r360_last_error()}")
                hs += (t1 - t0, t2 - t1, time.perf_counter() - t2, 1)
            rec[R_POSE:R_POSE + 16] = pose
            rec[R_INFO:R_INFO + 36] = info
            rec[R_STATUS] = 2 if self.stats[p].illposed else rc
            rec[R_SSO] = self.stats[p].sso
            rec[R_ERR] = self.stats[p].error
            fa, fb = fb, fa

    def _pipeline_queued(self, p: int, run: tuple[int, int], frames_of, out: np.ndarray, p0: int,
                         device_inputs: bool, repeats: int = 1):
        """_pipeline with the dense stage on the queue: submit pair i, then collect pair i-depth (so `depth`
        alignments per pipeline are in flight while the next frame is built and PbMap-registered).  Frames are
        built `lookahead` ahead of the pair in hand: iteration i enqueues frame i+L's build (L = lookahead) before
        RegisterPbMap(i, i+1) waits for frame i+1's planes, so with L = 2 the GPU works on frame i+2 while the host
        assembles and matches frame i+1's.  The upload of frame i+L+1 is issued right after frame i+L's build (same
        stream), so the next iteration's build does not wait for its copy.

        The `repeats` passes over the run are one stream of frame positions t = 0 .. repeats * (b - a + 1) - 1
        (frame a + t mod (b - a + 1); out[r] holds repeat r): a repeat's first frame is built while the previous
        repeat's last alignments are still in flight, instead of draining the pipeline at every repeat (a bubble
        that cost a 6-pair run about a tenth of its time).  No pair spans two repeats.  Position t lives in buffer
        t % nbuf, nbuf = depth + L + 2; before a buffer is refilled, every pair that used its previous frame is
        collected."""
        L = lib()
        ctx = self.ctxs[p]
        fr = self.frames[p]
        a, b = run
        q = self.queue
        hs = self.host_s[p]
        nfr = b - a + 1                  # frames per repeat
        T = nfr * repeats                # frame positions
        # shared run edges: position k = 0 of a repeat lives in this pipeline's edge buffer (left edge, built
        # here for the left neighbour too); k = nfr - 1 is the right neighbour's edge buffer (not built here)
        E = self.edges if self.share_edges else None
        left = E is not None and p > 0 and E[p]["shared"]
        right = E is not None and p + 1 < len(E) and E[p + 1]["shared"]

        def fidx(t):
            return a + t % nfr

        def buf(t):
            k = t % nfr
            if left and k == 0:
                return self.edge_frames[p]
            if right and k == nfr - 1:
                return self.edge_frames[p + 1]
            return fr[t % nbuf]

        def built_here(t):
            return not (right and t % nfr == nfr - 1)

        def load(t):
            if not built_here(t):
                return
            k, r = t % nfr, t // nfr
            if left and k == 0:
                # the left neighbour must be done with the previous repeat's copy, and so must this pipeline
                while pending and pending[0][1] <= t - nfr:
                    finish(*pending.pop(0))
                e = E[p]
                with e["cv"]:
                    if not e["cv"].wait_for(lambda: e["released"] >= r - 1 or e["failed"], EDGE_WAIT_S) or e["failed"]:
                        raise RuntimeError(f"pipeline {p}: left neighbour did not release edge frame {fidx(t)}")
            f, i = buf(t), fidx(t)
            if device_inputs:
                f.upload_device(*frames_of(i))
            else:
                f.upload_async(*frames_of(i))

        def build(t):
            if not built_here(t):
                return
            buf(t).build(self.flags, sync=False)
            if left and t % nfr == 0:
                e = E[p]
                with e["cv"]:
                    e["built"] = t // nfr
                    e["cv"].notify_all()

        def finish(ticket, t, st):
            rec = out[t // nfr][fidx(t) - p0]
            pose, info = np.zeros(16, np.float32), np.zeros(36, np.float32)
            if self.dense_only:
                dense = np.zeros(16, np.float32)
                rc = L.r360_dense_queue_collect(q.h, ticket, _fptr(dense), None, None, C.byref(st))
                if rc < 0:
                    raise RuntimeError(f"r360_dense_queue_collect: {L.r360_last_error()}")
                pose = (ROT_OFFSET_INV @ dense.reshape(4, 4).T.astype(np.float64) @ ROT_OFFSET).T.reshape(16)
                rc = 0
            else:
                rc = L.r360_register_collect(q.h, ticket, _fptr(pose), _fptr(info), C.byref(st))
                if rc < 0:
                    raise RuntimeError(f"r360_register_collect: {L.r360_last_error()}")
            rec[R_POSE:R_POSE + 16] = pose
            rec[R_INFO:R_INFO + 36] = info
            rec[R_STATUS] = 2 if st.illposed else rc
            rec[R_SSO] = st.sso
            rec[R_ERR] = st.error
            if right and t % nfr == nfr - 2:   # the last pair of a repeat: the right neighbour's edge is free again
                e = E[p + 1]
                with e["cv"]:
                    e["released"] = t // nfr
                    e["cv"].notify_all()

        nbuf = len(fr)
        pending = []
        LA = self.lookahead
        depth = nbuf - LA - 2
        last = T - 1
        for t in range(0, min(LA, last + 1)):   # positions 0 .. LA-1 built, position LA uploaded
            load(t)
            build(t)
        if LA <= last:
            load(LA)
        sts = [IcpStats() for _ in range(depth + 1)]
        n_sub = 0
        for t in range(0, last):
            t0 = time.perf_counter()
            # position t + LA + 1 refills the buffer of position u = t + LA + 1 - nbuf: collect the pairs (u - 1, u)
            # and (u, u + 1) that used it (without repeat boundaries the in-flight limit below already has)
            while pending and pending[0][1] <= t + LA + 1 - nbuf:
                finish(*pending.pop(0))
            cur, nxt = buf(t), buf(t + 1)
            if t + LA <= last:
                build(t + LA)   # its upload was issued one iteration earlier
            if t + LA + 1 <= last:
                load(t + LA + 1)
            t1 = time.perf_counter()
            if t % nfr == nfr - 1:   # the last frame of a repeat: no pair
                hs[0] += t1 - t0
                continue
            if not built_here(t + 1):   # the right neighbour's edge frame: built for this repeat?
                # collect the previous repeats' pairs first: the last of them releases the neighbour's edge for its
                # rebuild, which the neighbour may be waiting on (runs of at most `depth` pairs keep it pending here)
                while pending and pending[0][1] // nfr < (t + 1) // nfr:
                    finish(*pending.pop(0))
                e = E[p + 1]
                with e["cv"]:
                    if not e["cv"].wait_for(lambda: e["built"] >= (t + 1) // nfr or e["failed"], EDGE_WAIT_S) \
                            or e["built"] < (t + 1) // nfr:
                        raise RuntimeError(f"pipeline {p}: right neighbour did not build edge frame {fidx(t + 1)}")
            ticket = C.c_long()
            if self.dense_only:
                rc = L.r360_dense_queue_submit(q.h, cur.h, nxt.h, _fptr(self.eye), PHOTO_DEPTH, C.byref(self.params),
                                               C.byref(ticket))
            else:
                rc = L.r360_register_submit(ctx.h, q.h, cur.h, nxt.h, _fptr(self.eye), C.byref(self.params),
                                            self.max_match_planes, self.mode, C.byref(ticket))
            if rc != 0:
                raise RuntimeError(f"submit: {L.r360_last_error()}")
            t2 = time.perf_counter()
            pending.append((ticket.value, t, sts[n_sub % (depth + 1)]))
            n_sub += 1
            if len(pending) > depth:
                finish(*pending.pop(0))
            hs += (t1 - t0, t2 - t1, time.perf_counter() - t2, 1)
        t2 = time.perf_counter()
        while pending:
            finish(*pending.pop(0))
        hs[2] += time.perf_counter() - t2

    def run(self, p0: int, p1: int, frames_of, out: np.ndarray, repeats: int = 1, runs=None,
            device_inputs: bool = False):
        """Registers pairs [p0, p1) `repeats` times (out: (repeats, p1 - p0, REC)); frames_of(i) returns
        frame i's (bgr, depth) host arrays, which must outlive the call.  runs: the pipelines' pair runs
        (default: [p0, p1) split over the pipelines)."""
        runs = runs or split_range(p0, p1, self.P)
        assert len(runs) <= self.P

        body = self._pipeline_queued if self.queue else self._pipeline
        if self.share_edges:
            import threading
            # edge p (between runs p-1 and p, shared only where they meet): pipeline p has built its first frame
            # for repeat `built`; pipeline p-1 is done with it through repeat `released`
            self.edges = [None] + [{"cv": threading.Condition(), "built": -1, "released": -1, "failed": False,
                                     "shared": runs[q - 1][1] == runs[q][0]} for q in range(1, len(runs))]

        def worker(p):
            import threading
            self.native_ids.add(threading.get_native_id())
            if self.queue:   # the repeats as one stream of frames (no drain between them)
                try:
                    body(p, runs[p], frames_of, out, p0, device_inputs, repeats)
                except BaseException:
                    # a failed pipeline must not leave its neighbours waiting on its edges
                    for e in (self.edges or [])[p:p + 2]:
                        if e is not None:
                            with e["cv"]:
                                e["failed"] = True
                                e["cv"].notify_all()
                    raise
                return
            for r in range(repeats):
                body(p, runs[p], frames_of, out[r], p0, device_inputs)
        for f in [self.pool.submit(worker, p) for p in range(len(runs))]:
            f.result()
        for c in self.ctxs:
            c.sync()

    def close(self):
        self.pool.shutdown()
        if self.queue:
            self.queue.close()
        for fr in self.frames:
            for f in fr:
                f.close()
        for f in self.edge_frames or []:
            f.close()
        for c in self.cals:
            c.close()
        for c in self.ctxs:
            c.close()
