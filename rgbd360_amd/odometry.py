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

import numpy as np

from . import (PLANAR_3DoF, Calib360, Context, DenseQueue, Frame360, IcpParams, EXTRINSICS_DIR, C, _check, lib)

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


def stream_pieces(p0: int, p1: int, repeats: int, P: int) -> list[list[tuple[int, int, int]]]:
    """How r360_sequence_run cuts the repeats x (p1 - p0) pair registrations (repeat-major) into P contiguous pieces:
    per piece its segments (repeat, first pair, last pair + 1).  Each segment costs one frame build beyond its pairs."""
    n = p1 - p0
    total = repeats * n
    parts = min(P, total)
    out, at = [], 0
    for k in range(parts):
        e = at + total // parts + (1 if k < total % parts else 0)
        segs, u = [], at
        while u < e:
            r, i = divmod(u, n)
            b = min(n, i + (e - u))
            segs.append((r, p0 + i, p0 + b))
            u += b - i
        out.append(segs)
        at = e
    return out


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


class SequenceParams(C.Structure):
    """r360_sequence_params (include/rgbd360_hip.h)."""
    _fields_ = [("rows", C.c_int), ("cols", C.c_int), ("pipelines", C.c_int), ("queue", C.c_int), ("depth", C.c_int),
                ("lookahead", C.c_int), ("plane_batch", C.c_int), ("workload", C.c_int),
                ("max_match_planes", C.c_size_t), ("mode", C.c_int), ("icp", IcpParams)]


SEQ_FULL, SEQ_PLANES, SEQ_DENSE = 0, 1, 2


class SequenceRunner:
    """P pipelines on one GPU: the C++ sequence runner of the library (r360_sequence, host/sequence.cpp), each
    pipeline a host thread of the library with its own r360_ctx (HIP stream + device GN state) and ring of Frame360
    buffers.  This class only passes the frames' image pointers in and the pair records out.

    queue > 0: the pipelines' alignFrames360 calls go to one dense queue (r360_dense_queue, batches of up to
    `queue` pairs per launch); each pipeline keeps `depth` alignments in flight while it builds (`lookahead` frames
    ahead) and PbMap-registers the next frames.  Records are batch-invariant (bit-identical for any cut into pipelines,
    batches and ranks); against the unqueued run (lone alignments, two workgroups per CU) the PbMap stage is identical
    and the poses equal to rounding (tests/test_gpu_sequence.py).

    Attributes mirror the pipelines: ctxs / cals / frames (non-owning views of each pipeline's context, calibration
    and frame ring), queue (the dense queue's view, or None), host_s ([P, 4] host seconds: load + build enqueue,
    PbMap stage, dense wait, pairs) and native_ids (the pipeline threads' OS ids)."""

    def __init__(self, device: int, rows: int, cols: int, pipelines: int, params: IcpParams,
                 planes: bool = True, max_match_planes: int = 25, mode: int = PLANAR_3DoF, dense_only: bool = False,
                 queue: int = 0, planes_only: bool = False, depth: int = 1, lookahead: int = 1,
                 plane_batch: int | None = None):
        L = lib()
        sp = SequenceParams()
        L.r360_sequence_default_params(C.byref(sp))
        sp.rows, sp.cols, sp.pipelines = rows, cols, pipelines
        sp.queue = 0 if planes_only else queue
        sp.depth, sp.lookahead = max(1, depth), max(1, lookahead)
        if plane_batch is not None:
            sp.plane_batch = plane_batch
        sp.workload = SEQ_PLANES if planes_only else SEQ_DENSE if dense_only or not planes else SEQ_FULL
        sp.max_match_planes, sp.mode = max_match_planes, mode
        sp.icp = params
        h = C.c_void_p()
        _check(L.r360_sequence_create(device, C.byref(sp), EXTRINSICS_DIR.encode(), C.byref(h)), "r360_sequence_create")
        self.h, self.P, self.params = h, pipelines, params
        self.lookahead = sp.lookahead
        self.dense_only, self.planes_only = sp.workload == SEQ_DENSE, sp.workload == SEQ_PLANES
        q = C.c_void_p()
        _check(L.r360_sequence_info(h, None, C.byref(q)), "r360_sequence_info")
        self.queue = DenseQueue._view(q, device) if q.value else None
        self.ctxs, self.cals, self.frames, self.native_ids = [], [], [], set()
        for p in range(pipelines):
            cx, ca, n, tid = C.c_void_p(), C.c_void_p(), C.c_int(), C.c_long()
            fr = (C.c_void_p * 16)()
            _check(L.r360_sequence_pipeline(h, p, C.byref(cx), C.byref(ca), fr, 16, C.byref(n), C.byref(tid)),
                   "r360_sequence_pipeline")
            ctx = Context._view(cx, device)
            cal = Calib360._view(ca, ctx, rows, cols)
            self.ctxs.append(ctx)
            self.cals.append(cal)
            self.frames.append([Frame360._view(C.c_void_p(fr[k]), cal) for k in range(min(n.value, 16))])
            self.native_ids.add(tid.value)
        self.host_s = np.zeros((pipelines, 4))
        pc = C.c_void_p()
        _check(L.r360_sequence_plane_stats(h, None, None, None, C.byref(pc)), "r360_sequence_plane_stats")
        self.plane_ctx = Context._view(pc, device) if pc.value else None
        self.host_detail = np.zeros((pipelines, 4))   # build enqueue, upload enqueue, refill collects, edge waits

    def run(self, p0: int, p1: int, frames_of, out: np.ndarray, repeats: int = 1, runs=None,
            device_inputs: bool = False):
        """Registers pairs [p0, p1) `repeats` times (out: (repeats, p1 - p0, REC) float32); frames_of(i) returns
        frame i's (bgr, depth): host arrays, which must outlive the call, or with device_inputs device pointers of
        images resident in HBM.  The repeats x (p1 - p0) registrations form one stream cut into contiguous pieces, one
        per pipeline; runs (optional): pair runs tiling [p0, p1), pipeline k taking run k of every repeat instead."""
        assert (runs is None or len(runs) <= self.P) and out.dtype == np.float32 and out.flags.c_contiguous
        assert out.shape[0] >= repeats and out.shape[1] == p1 - p0 and out.shape[2] == REC
        n = p1 - p0 + 1
        bgr, dep = (C.c_void_p * n)(), (C.c_void_p * n)()
        keep = []
        for k in range(n):
            b, d = frames_of(p0 + k)
            if b is None or d is None:   # null image pointers: the library fails the run (failure-path tests)
                bgr[k], dep[k] = None, None
            elif device_inputs:
                bgr[k], dep[k] = int(b), int(d)
            else:
                assert b.dtype == np.uint8 and d.dtype == np.uint16 and b.flags.c_contiguous and d.flags.c_contiguous
                keep.append((b, d))
                bgr[k], dep[k] = b.ctypes.data, d.ctypes.data
        rv = np.asarray(runs if runs else [(0, 0)], np.int32).reshape(-1)
        L = lib()
        rc = L.r360_sequence_run(self.h, p0, p1, bgr, dep, int(device_inputs), repeats, rv.ctypes.data,
                                 len(runs) if runs else 0, out.ctypes.data)
        hs = np.zeros(8 * self.P)
        L.r360_sequence_host_times(self.h, hs.ctypes.data, 1)
        self.host_s += hs.reshape(self.P, 8)[:, :4]
        self.host_detail += hs.reshape(self.P, 8)[:, 4:]
        if rc != 0:
            raise RuntimeError(f"r360_sequence_run: {L.r360_last_error().decode()}")

    def plane_stats(self):
        """The plane queue's {batches, frames, max_batch} so far (zeros without one)."""
        b, f, m = C.c_long(), C.c_long(), C.c_int()
        _check(lib().r360_sequence_plane_stats(self.h, C.byref(b), C.byref(f), C.byref(m), None), "plane_stats")
        return {"batches": b.value, "frames": f.value, "max_batch": m.value}

    def close(self):
        if self.h:
            lib().r360_sequence_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
