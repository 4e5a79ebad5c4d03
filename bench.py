"""bench.py — registered Frame360 pairs/sec on MI355X (BASELINE.json metric) + ICP-reduce roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload sequence|dense]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload "sequence" (default; BASELINE.json configs[3], whose per-pair work is configs[1] + configs[2]):
OdometryRGBD360 over the synthetic 256-frame sequence (procedural room, seed 360, 8 x 480x640 sensors).
One step registers each of the 255 consecutive pairs exactly once (rgbd360_amd/odometry.py):
  * the pairs are split contiguously over the ranks (one process per GPU) and, within a rank, over P
    pipelines (host thread + HIP stream each, running free);
  * per pair the new frame's raw 8-sensor images are uploaded from page-locked host memory (inside the
    timed region, BASELINE.md §3 "from input upload"), the Frame360 is built on the GPU (undistort, cloud
    + 2x2 median downsample, bilateral filter, normals, plane segmentation + refinement, PbMap
    descriptors and grouping, spherical stitch, 5-level pyramid with gradients), then
    RegisterRGBD360::RegisterPbMap(25 planes, PLANAR_3DoF) and RegisterPhotoICP::alignFrames360(PHOTO_DEPTH)
    initialised with the rotOffset-conjugated PbMap pose (OdometryKeyFrame360.cpp:205-254): the reference
    schedule on levels 4..1 and exactly 20 Gauss-Newton iterations at level 0 (timing mode);
  * the per-pair records {pose, information, status, SSO, error} of every rank are gathered with one RCCL
    all_gather over xGMI and rank 0 composes the trajectory (OdometryRGBD360.cpp:257) — inside the timed
    region.
Strong scaling: the sequence is the same at every N.  Workload "dense" (configs[2]; configs[4] with
--rows 960 --cols 1280 --iters0 50): stitch + pyramid of every frame and alignFrames360 per pair, no planes.

Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Hardware queues per process: 16 only where the environment leaves GPU_MAX_HW_QUEUES unset.  The GPU box
# presets 4 (HIP's default), so the driver's bench lines run with a pool of 4 pooled queues (the line records the
# value in config.gpu_max_hw_queues); the dense queue and the plane queue have CU-masked hardware queues of their
# own outside the pool, and 4 vs 16 pooled queues measured within 1 % (profiles/r5_envab/).
# Must precede HIP initialisation.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

METRIC = "registered Frame360 pairs/sec @ 8×640×480; ICP-reduce HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
SEED = 360 << 16
ICP_SOURCES = ["rgbd360_amd/csrc/kernels/icp_kernels.hip", "rgbd360_amd/csrc/kernels/icp_common.inc",
               "rgbd360_amd/csrc/kernels/icp_gn.inc", "rgbd360_amd/csrc/kernels/icp_la.inc",
               "rgbd360_amd/csrc/libm_f32.h", "rgbd360_amd/csrc/r360_internal.h"]


def _sha16(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def icp_source_hash():
    """Hash of the ICP pass's sources: a profile's PMC traffic is reported only for the kernel it measured."""
    h = hashlib.sha256()
    for p in ICP_SOURCES:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def gather_records(allgather, rec, pad_to):
    """Every rank's pair records (K, n, REC), padded to the largest shard and all-gathered in one call (RCCL
    over xGMI through rgbd360_amd.Comm on the GPU; gloo in the CPU tests).  Returns the records of the whole
    sequence in rank order and the shard sizes."""
    k, n, w = rec.shape
    buf = np.zeros((k, pad_to, w), np.float32)
    buf[:, :n] = rec
    buf[:, :, w - 1] = n                # the record's last slot is unused: it carries the shard size
    allr = allgather(buf)               # (world, K, pad, REC)
    sizes = [int(x[0, 0, w - 1]) for x in allr]
    return np.concatenate([x[:, :m] for x, m in zip(allr, sizes)], axis=1), sizes


class RankGroup:
    """One process per GPU: torch.distributed's gloo group (host only, never touches the GPU) for the
    rendezvous and barriers, and an RCCL communicator of the library (rgbd360_amd.Comm) for the device
    collectives over xGMI."""

    def __init__(self, device, rehearsal=False):
        import torch.distributed as dist
        import rgbd360_amd as R
        dist.init_process_group("gloo")
        self.dist = dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.comm = None
        if not rehearsal:
            uid = [R.Comm.unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            self.comm = R.Comm(device, self.world, self.rank, uid[0])

    def barrier(self, ctxs=()):
        for c in ctxs:
            c.sync()
        self.dist.barrier()

    def allgather(self, a):
        if self.comm is not None:
            return self.comm.allgather(a)
        import torch     # rehearsal of N ranks on one GPU (R360_BENCH_REHEARSAL=1): host gloo gather
        t = torch.from_numpy(np.ascontiguousarray(a))
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return np.stack([o.numpy() for o in out])

    def max(self, v):
        if self.comm is not None:
            return self.comm.allreduce_max(v)
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.comm is not None:
            self.comm.close()
        self.dist.destroy_process_group()


def thread_cpu_s():
    """CPU seconds (user + system) per live OS thread of this process: {tid: seconds}."""
    out = {}
    tck = os.sysconf("SC_CLK_TCK")
    for t in os.listdir("/proc/self/task"):
        try:
            f = open(f"/proc/self/task/{t}/stat").read()
            fields = f[f.rindex(")") + 2:].split()
            out[int(t)] = (int(fields[11]) + int(fields[12])) / tck
        except (OSError, ValueError, IndexError):
            pass
    return out


def host_cpu_info():
    """Host cores usable by this process (affinity and cgroup quota) and the CPU model string."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"affinity": aff, "cgroup_quota": quota, "usable": min(aff, quota) if quota else aff, "model": model}


def cpu_baseline(cal, frames_of, first, last, workload, iters0, budget_s=10.0):
    """The CPU oracle (C++ restatement, OpenMP where the reference parallelises: the 8 sensors, the ICP
    rows) on a bounded sample of the same workload: consecutive pairs of the same synthetic sequence,
    each = PbMap build of the new frame + RegisterPbMap + stitch + alignFrames360.  Timed at 8 threads
    (the reference's num_threads(8), Frame360.h:620) and at every usable host core."""
    from oracle import oracle360 as O
    rt, rti, K = cal.extrinsics()
    Km = K.reshape(3, 3).T
    rt8 = np.stack([rt[16 * k:16 * k + 16].reshape(4, 4).T for k in range(8)])
    prm = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255), fixed_iters_level0=iters0)
    a = np.float64(np.float32(157.5)) * 3.14159265359 / 180
    Ro = np.eye(4, dtype=np.float32)
    Ro[1, 1] = Ro[2, 2] = np.float32(np.cos(a))
    Ro[1, 2], Ro[2, 1] = np.float32(np.sin(a)), -np.float32(np.sin(a))
    Ri = Ro.T.copy()

    def build(i):
        b, d = frames_of(i)
        sb, sd = O.stitch(b, d, rti, Km)
        pm = O.PbMap(d.astype(np.float32) * np.float32(0.001), b, rt8) if workload == "sequence" else None
        return sb, sd, pm

    gomp = None
    try:
        gomp = ctypes.CDLL("libgomp.so.1")
    except OSError:
        pass
    info = host_cpu_info()
    runs = []
    for threads in sorted({min(8, info["usable"]), info["usable"]}):
        if gomp is not None:
            gomp.omp_set_num_threads(threads)
        prev = build(first)
        n, t0 = 0, time.perf_counter()
        while True:
            cur = build(first + n + 1)
            if workload == "sequence":
                r = O.register_pbmap(prev[2], cur[2], 25, O.PLANAR_3DoF)
                init = Ro @ (r["pose"] if r["good"] else np.eye(4, dtype=np.float32)) @ Ri
            else:
                init = None
            O.align360(prev[0], prev[1], cur[0], cur[1], init, O.PHOTO_DEPTH, prm)
            prev = cur
            n += 1
            if time.perf_counter() - t0 > budget_s or first + n + 1 > last:
                break
        dt = time.perf_counter() - t0
        runs.append({"threads": threads, "value": n / dt, "pairs": n, "seconds": round(dt, 2)})
    what = ("PbMap build of the new frame + RegisterPbMap + stitch + alignFrames360" if workload == "sequence"
            else "stitch + alignFrames360")
    best = max(runs, key=lambda r: r["value"])
    return {"value": best["value"], "unit": "pairs/s", "cores": best["threads"], "kind": "port",
            "runs": runs, "cpu_model": info["model"], "host_cores": info,
            "sample": f"consecutive synthetic pairs from frame {first} of the same sequence ({what}, nPyr=5, "
                      f"{iters0} level-0 iterations), oracle/liboracle360.so (g++ -O3 -fopenmp), ~{budget_s:.0f} s per "
                      "thread count; value = the faster run"}


def config1_leg(device, reps=5):
    """BASELINE configs[0]: RegisterPairRGBD360 on the reference's sample captures sphere_images_1.bin vs _10.bin
    (Registration/RegisterPairRGBD360.cpp:72-95: two Frame360 loads, undistort, buildSphereCloud + getPlanes, then
    RegisterPbMap(25 planes, PLANAR_3DoF)), per stage, median of `reps` runs after one warm-up.  The CPU leg is the
    oracle (OpenMP at the reference's 8 threads, Frame360.h:620); the GPU leg is the same stages through the library
    (Frame360 load + upload, plane build incl. the host PbMap assembly, RegisterPbMap)."""
    import rgbd360_amd as R
    from oracle import oracle360 as O
    paths = [os.path.join(R.SAMPLES_DIR, f"sphere_images_{k}.bin") for k in (1, 10)]
    rt8 = O.read_extrinsics(R.EXTRINSICS_DIR)
    clams = [O.Clams(os.path.join(R.INTRINSICS_DIR, f"distortion_model{k + 1}.r360")) for k in range(8)]
    gomp = None
    try:
        gomp = ctypes.CDLL("libgomp.so.1")
        gomp.omp_set_num_threads(8)
    except OSError:
        pass
    cpu = {k: [] for k in ("loadFrame", "undistort", "getPlanes", "RegisterPbMap", "total")}
    r = None
    for it in range(reps + 1):
        t = [time.perf_counter()]
        raw = [O.load_bin(pth) for pth in paths]
        t.append(time.perf_counter())
        dm = [np.stack([clams[k].undistort(O.depth_to_m(d[k])) for k in range(8)]) for _, d in raw]
        t.append(time.perf_counter())
        maps = [O.PbMap(m, b, rt8) for m, (b, _) in zip(dm, raw)]
        t.append(time.perf_counter())
        r = O.register_pbmap(maps[0], maps[1], 25, O.PLANAR_3DoF)
        t.append(time.perf_counter())
        if it:
            for k, name in enumerate(("loadFrame", "undistort", "getPlanes", "RegisterPbMap")):
                cpu[name].append((t[k + 1] - t[k]) * 1e3)
            cpu["total"].append((t[-1] - t[0]) * 1e3)
    ctx = R.Context(device)
    cal = R.Calib360(ctx, 240, 320)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    cal.loadIntrinsicCalibration(R.INTRINSICS_DIR)
    frames = [R.Frame360(cal), R.Frame360(cal)]
    reg = R.RegisterRGBD360(ctx)
    gpu = {k: [] for k in ("loadFrame", "undistort+getPlanes", "RegisterPbMap", "total")}
    good, matches = None, None
    for it in range(reps + 1):
        t = [time.perf_counter()]
        for f, pth in zip(frames, paths):
            f.loadFrame(pth)
        ctx.sync()
        t.append(time.perf_counter())
        for f in frames:
            f.build(R.BUILD_UNDISTORT | R.BUILD_PLANES, sync=False)
        for f in frames:
            f.planes()
        t.append(time.perf_counter())
        good = reg.RegisterPbMap(frames[0], frames[1], 25, R.PLANAR_3DoF)
        matches = reg.getMatchedPlanes()
        t.append(time.perf_counter())
        if it:
            for k, name in enumerate(("loadFrame", "undistort+getPlanes", "RegisterPbMap")):
                gpu[name].append((t[k + 1] - t[k]) * 1e3)
            gpu["total"].append((t[-1] - t[0]) * 1e3)
    for f in frames:
        f.close()
    cal.close()
    ctx.close()
    med = lambda d: {k: round(float(np.median(v)), 3) for k, v in d.items()}
    return {"workload": "config1: RegisterPairRGBD360 on samples/sphere_images_1.bin vs _10.bin (QVGA 8x240x320, CLAMS + "
                        "Rt calibration): 2 x (loadFrame, undistort, buildSphereCloud + getPlanes) + RegisterPbMap(25, "
                        "PLANAR_3DoF)",
            "cpu_ms": med(cpu), "cpu_threads": 8, "cpu_kind": "port (oracle/liboracle360.so)",
            "gpu_ms": med(gpu), "runs": reps,
            "pbmap_good": bool(good), "matches": len(matches or {}), "oracle_matches": len(r["matches"]),
            "same_matches": bool(matches == r["matches"])}


def sequential_leg(device, rows, cols, p0, frames_of, params, pairs=32, plane_batch=0):
    """The reference's sequential caller (Registration/OdometryRGBD360.cpp:141-257): one pair at a time through the
    C++ sequence runner with one pipeline and no dense queue (upload + build of the new frame, Register() on the
    pipeline's own stream, wait), over `pairs` consecutive pairs of the same sequence.  plane_batch 0: the plane stage
    on the pipeline's own stream (a lone frame has nothing to batch with); since the waiting thread assembles the new
    frame's PbMap itself (round 6, pbmap.cpp planes_join) that is 2.22 ms per pair against 2.32 through a plane queue
    (None: the runner's default, profiles/r6_seq).  Returns the rate and the per-pair host split (load + build
    enqueue, the PbMap stage with its waits, the dense wait)."""
    from rgbd360_amd import odometry as OD
    runner = OD.SequenceRunner(device, rows, cols, 1, params, queue=0, plane_batch=plane_batch)
    try:
        runner.run(p0, p0 + 4, frames_of, np.zeros((1, 4, OD.REC), np.float32))   # warm-up
        rec = np.zeros((1, pairs, OD.REC), np.float32)
        runner.host_s[:] = 0
        runner.host_detail[:] = 0
        for c in runner.ctxs:
            c.host_times(reset=True)
        t0 = time.perf_counter()
        runner.run(p0, p0 + pairs, frames_of, rec)
        dt = time.perf_counter() - t0
        hs = runner.host_s.sum(axis=0)
        ht = np.sum([c.host_times() for c in runner.ctxs], axis=0)
        split = {k: round(1e3 * v / pairs, 3) for k, v in
                 zip(("load_build_enqueue", "pbmap_stage", "dense_wait"), hs[:3])}
        hd = runner.host_detail.sum(axis=0)   # inside load_build_enqueue
        split.update({"upload_enqueue": round(1e3 * hd[1] / pairs, 3), "build_enqueue": round(1e3 * hd[0] / pairs, 3)})
        split.update({k: round(1e3 * v / max(ht[3], 1), 3) for k, v in
                      zip(("pbmap_wait_frames", "pbmap_match_tables", "pbmap_tree_pose"), ht[:3])})
    finally:
        runner.close()
    return {"value": pairs / dt, "unit": "pairs/s", "ms_per_pair": dt / pairs * 1e3, "pairs": pairs,
            "plane_batch": plane_batch, "host_ms_per_pair": split,
            "workload": "config4's pairs one at a time (C++ runner, 1 pipeline, no dense queue): upload, Frame360 build, "
                        "Register() per pair, as OdometryRGBD360.cpp:141-257 calls it"}


def half_leg(kind, device, rows, cols, p0, p1, frames_of, params, pipelines, queue, depth, repeats=3):
    """BASELINE configs[1] / configs[2] as secondary blocks of the default line: one half of the headline workload
    over the same synthetic sequence, same pipelines, batched like the headline run.
      kind "planes" (configs[1]): per pair the upload + Frame360 build with planes (PbMap) + RegisterPbMap(25,
                                  PLANAR_3DoF), no alignFrames360;
      kind "dense"  (configs[2]): per pair the upload + stitch + 5-level pyramid + alignFrames360(PHOTO_DEPTH) with
                                  the reference schedule on levels 4..1 and exactly params.fixed_iters_level0 (20) GN
                                  iterations at level 0, the dense queue batching the pipelines' alignments.
    Returns pairs/s (whole sequence x repeats after one warm-up pass) and, for the dense half, its level-0 pass."""
    from rgbd360_amd import odometry as OD
    P = min(pipelines, p1 - p0)
    # the plane half alone runs every pipeline's plane stage on its own stream: with no dense half competing for the
    # GPU, twelve concurrent chains beat batches on the plane queue (2759 vs 2289 pairs/s, profiles/r5_planes)
    runner = OD.SequenceRunner(device, rows, cols, P, params, planes=kind == "planes",
                               dense_only=kind == "dense", queue=queue, planes_only=kind == "planes", depth=depth,
                               plane_batch=0 if kind == "planes" else None)
    runner.run(p0, p1, frames_of, np.zeros((1, p1 - p0, OD.REC), np.float32), repeats=1)   # warm-up
    qctx = runner.queue.ctx if runner.queue else None
    if qctx:
        qctx.kernel_time_reset()
    rec = np.zeros((repeats, p1 - p0, OD.REC), np.float32)
    t0 = time.perf_counter()
    runner.run(p0, p1, frames_of, rec, repeats=repeats)
    elapsed = time.perf_counter() - t0
    out = {"value": (p1 - p0) * repeats / elapsed, "unit": "pairs/s", "pairs": p1 - p0, "repeats": repeats,
           "ms_per_pair": elapsed / ((p1 - p0) * repeats) * 1e3, "pipelines": P}
    if kind == "planes":
        st = rec[-1, :, OD.R_STATUS]
        out["workload"] = ("config2 over the config4 sequence: per pair upload + Frame360 build with planes (PbMap) + "
                           "RegisterPbMap(25 planes, PLANAR_3DoF), no alignFrames360")
        out["pbmap_failed"] = int((st == 1).sum())
    else:
        # unqueued runs (--queue 0: each pipeline aligns on its own context) have no shared in-kernel statistics
        us, n, nj = qctx.kernel_stats(0) if qctx else (0.0, 0, 0)
        W0 = rows * 8                       # sphere width: 8 sensors of `rows` (the sensors are mounted sideways)
        N0 = int(W0 * 0.5 * 60.0 / 180) * W0
        sso = float(np.mean(rec[:, :, OD.R_SSO]))
        alg = 8.0 * N0 + 24.0 * sso * N0
        avg_ms = us / max(n, 1) * 1e-3
        ppl = nj / max(n, 1)
        ach = ppl * alg / (avg_ms * 1e-3) / 1e9 if n else None
        out["workload"] = ("config3 over the config4 sequence: per pair upload, stitch + 5-level pyramid, "
                           f"alignFrames360(PHOTO_DEPTH) levels 4..1 reference schedule + {params.fixed_iters_level0} GN "
                           "iterations at level 0 (dense queue batches of up to 16 pairs)")
        # the same kernel on the same frame size as the headline: its PMC profile's HBM bytes per pair-pass apply,
        # scaled to this leg's pairs per launch (when the profile measured the current ICP sources)
        traffic, tsrc = None, None
        tf = os.path.join(ROOT, "profiles", "latest", "l0_pass.json")
        if n and (rows, cols) == (480, 640) and os.path.exists(tf):
            prof = json.load(open(tf))
            if prof.get("icp_source_hash") == icp_source_hash() and prof.get("hbm_bytes_per_pair_pass"):
                traffic, tsrc = prof["hbm_bytes_per_pair_pass"] * ppl, prof.get("tag")
        out["roofline"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": (ach / HBM_PEAK_GBS) if ach else None, "traffic": traffic,
                           "traffic_profile": tsrc, "avg_launch_ms": avg_ms, "launches": n,
                           "pairs_per_launch": ppl, "bytes_per_pair_pass": alg,
                           "kernel": "k_icp_pass<PHOTO_DEPTH> (level 0)", "timing": "in-kernel execution span"}
    runner.close()
    return out


def config5_leg(device, rt8, pairs=48, iters0=50, pipelines=8, depth=2, repeats=3):
    """BASELINE configs[4], the HBM stress case, as a secondary block of the default line: the dense stage
    (upload, stitch + 5-level pyramid, alignFrames360(PHOTO_DEPTH) with the reference schedule on levels 4..1
    and exactly `iters0` GN iterations at level 0) over `pairs` consecutive pairs of the synthetic sequence at
    8 x 1280x960 (1280 x 7680 sphere), batched like the headline run (pipelines x depth alignments in flight on
    the dense queue).  Its level-0 working set (~268 MB per pair-pass) exceeds the 256 MB Infinity Cache, so
    this is the one configuration whose roofline is an HBM roofline."""
    import rgbd360_amd as R
    from rgbd360_amd import odometry as OD
    rows, cols = 960, 1280
    t_gen = time.perf_counter()
    nf = pairs + 1
    BGR = np.zeros((nf, 8, rows, cols, 3), np.uint8)
    DEP = np.zeros((nf, 8, rows, cols), np.uint16)
    for j in range(nf):
        BGR[j], DEP[j] = R.synth_frame_rt(rows, cols, rt8, SEED, R.synth_path_pose(SEED, j))
    gen_s = time.perf_counter() - t_gen
    pinned = R.HostPinned(BGR, DEP)
    params = R.IcpParams.default()
    params.n_pyr = 5
    params.std_dev_photo = np.float32(3.0 / 255)
    params.fixed_iters_level0 = iters0
    runner = OD.SequenceRunner(device, rows, cols, pipelines, params, planes=False, dense_only=True, queue=16,
                               depth=depth)

    def frames_of(i):
        return BGR[i], DEP[i]
    runner.run(0, pairs, frames_of, np.zeros((1, pairs, OD.REC), np.float32), repeats=1)   # warmup
    qctx = runner.queue.ctx
    q0 = runner.queue.stats()
    qctx.kernel_time_reset()
    rec = np.zeros((repeats, pairs, OD.REC), np.float32)
    t0 = time.perf_counter()
    runner.run(0, pairs, frames_of, rec, repeats=repeats)
    elapsed = time.perf_counter() - t0
    us, n, nj = qctx.kernel_stats(0)
    q1 = runner.queue.stats()
    runner.close()
    pinned.close()
    W0 = rows * 8
    H0 = int(W0 * 0.5 * 60.0 / 180)
    N0 = H0 * W0
    sso = float(np.mean(rec[:, :, OD.R_SSO]))
    alg = 8.0 * N0 + 24.0 * sso * N0
    avg_ms = us / max(n, 1) * 1e-3
    ppl = nj / max(n, 1)
    ach = ppl * alg / (avg_ms * 1e-3) / 1e9 if n else None
    # HBM bytes per level-0 launch from the HiRes rocprofv3 --pmc passes (tools/prof_r3.sh, tools/hires_summary.py,
    # profiles/latest/hires_pmc.json), reported only when that profile measured the current ICP sources
    traffic, traffic_src = None, None
    hf = os.path.join(ROOT, "profiles", "latest", "hires_pmc.json")
    if os.path.exists(hf):
        prof = json.load(open(hf))
        if prof.get("icp_source_hash") == icp_source_hash() and prof.get("hbm_bytes_per_pair_pass"):
            traffic, traffic_src = prof["hbm_bytes_per_pair_pass"] * ppl, prof.get("tag", "latest/hires_pmc.json")
    # per-pair accuracy against the synthetic ground truth (the dense stage starts from identity)
    gt = [R.synth_path_pose(SEED, k).astype(np.float64) for k in range(nf)]
    rot_err = []
    for i in range(pairs):
        G = np.linalg.inv(gt[i]) @ gt[i + 1]
        D = np.linalg.inv(G) @ rec[-1, i, OD.R_POSE:OD.R_POSE + 16].reshape(4, 4).T.astype(np.float64)
        rot_err.append(float(np.degrees(np.arccos(np.clip((np.trace(D[:3, :3]) - 1) / 2, -1, 1)))))
    return {
        "workload": (f"config5: synthetic 8x{cols}x{rows} sequence, {pairs} consecutive pairs x {repeats} repeats; per "
                     f"pair: upload, stitch + 5-level pyramid, alignFrames360(PHOTO_DEPTH) levels 4..1 reference "
                     f"schedule + {iters0} GN iterations at level 0 ({pipelines} pipelines x {depth} in flight, dense "
                     "queue batches of up to 16 pairs)"),
        "sphere": f"{H0}x{W0}", "value": pairs * repeats / elapsed, "unit": "pairs/s",
        "ms_per_pair": elapsed / (pairs * repeats) * 1e3,
        "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (ach / HBM_PEAK_GBS) if ach else None, "traffic": traffic,
                     "traffic_profile": traffic_src, "traffic_per_pair_pass": (traffic / ppl) if traffic else None,
                     "kernel": "k_icp_pass<PHOTO_DEPTH> (level 0)", "avg_launch_ms": avg_ms, "launches": n,
                     "pairs_per_launch": ppl, "bytes_per_pair_pass": alg, "visible_frac": sso,
                     "timing": "in-kernel execution span (s_memrealtime) of every level-0 launch of the timed repeats"},
        "dense_queue": {"batches": q1["batches"] - q0["batches"], "jobs": q1["jobs"] - q0["jobs"]},
        "max_pair_rot_err_deg": max(rot_err), "frame_generation_s": round(gen_s, 1),
    }


def main(argv=None, runner_factory=None):
    """argv: the command line (sys.argv[1:] by default).  runner_factory(device, rows, cols, P, params, **kw): the
    pipelines' runner (odometry.SequenceRunner by default; the CPU tests pass a stand-in that fills the pair records
    without a GPU, to drive this function's shard / gather / max-over-ranks / composition path over gloo)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows", type=int, default=480)
    ap.add_argument("--cols", type=int, default=640)
    ap.add_argument("--iters0", type=int, default=20)
    ap.add_argument("--frames", type=int, default=256, help="sequence length (frames)")
    ap.add_argument("--workload", choices=["sequence", "dense", "planes"], default="sequence")
    ap.add_argument("--streams", type=int, default=12, help="max pipelines per GPU (host thread + HIP stream each; "
                    "12 with the batched plane stage: 1472-1477 vs 1437-1458 pairs/s at 10, profiles/r5_pq2/)")
    ap.add_argument("--min-run", type=int, default=6,
                    help="with --per-step-runs: min pairs per pipeline run (each run rebuilds a halo frame)")
    ap.add_argument("--per-step-runs", action="store_true",
                    help="split each step's pairs into one run per pipeline (rounds 2-4) instead of cutting the steps x "
                         "pairs stream into one contiguous piece per pipeline (default)")
    ap.add_argument("--stage-timing", action="store_true",
                    help="diagnostic: HIP events around EVERY launch of the timed run (per-stage times; slows the run)")
    ap.add_argument("--queue", type=int, default=16,
                    help="dense queue batch size (alignFrames360 of up to N pairs per launch); 0 = one launch per pair "
                         "on each pipeline's stream")
    ap.add_argument("--depth", type=int, default=3,
                    help="dense queue: alignments in flight per pipeline (each needs one more Frame360 buffer)")
    ap.add_argument("--lookahead", type=int, default=1,
                    help="dense queue: frames whose build is enqueued ahead of the pair being registered")
    ap.add_argument("--plane-batch", type=int, default=8,
                    help="plane stages of up to N frames per launch on one stream (0: each pipeline builds its frames' "
                         "planes on its own stream)")
    ap.add_argument("--emulate", type=str, default=None,
                    help="RANK/WORLD: run that rank's shard alone (single-GPU rehearsal of an N-GPU shard)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-resident", action="store_true", help="skip the HBM-resident-input secondary run")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 (8x1280x960, 50 iterations) leg")
    ap.add_argument("--no-halves", action="store_true", help="skip the config-2 (planes) and config-3 (dense) legs")
    ap.add_argument("--no-isolated", action="store_true",
                    help="skip the lone-pipeline rerun after the timed region (profiling: the trace then holds only "
                         "the warmup and timed launches)")
    ap.add_argument("--eval-probe", action="store_true", help="diagnostic: also time the level-0 pass in eval mode")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rehearsal = os.environ.get("R360_BENCH_REHEARSAL") == "1"   # N ranks sharing one GPU (gloo records)
    if rehearsal:
        local = 0
    group = RankGroup(local, rehearsal) if world > 1 else None
    shard_rank, shard_world = rank, world
    if args.emulate:
        shard_rank, shard_world = (int(x) for x in args.emulate.split("/"))

    import rgbd360_amd as R
    from rgbd360_amd import odometry as OD

    p0, p1 = OD.shard_pairs(shard_rank, shard_world, args.frames)
    # the steps x shard pairs form one stream, cut into one contiguous piece per pipeline (each piece rebuilds the
    # first frame of each of its segments: a few extra frame builds per step, no coupling between pipelines)
    if args.per_step_runs:
        runs = OD.split_range(p0, p1, OD.pipelines_for(p1 - p0, args.streams, args.min_run))
        P = len(runs)
    else:
        runs = None
        P = max(1, min(args.streams, (p1 - p0) * max(args.steps, 1)))

    # raw frames p0..p1 of this rank, rendered on the host, in page-locked memory (uploaded per pair
    # inside the timed region)
    t_gen = time.perf_counter()
    rt8 = np.stack([np.loadtxt(os.path.join(R.EXTRINSICS_DIR, f"Rt_0{k + 1}.txt"), dtype=np.float32)
                    for k in range(8)])
    nf = p1 - p0 + 1
    BGR = np.zeros((nf, 8, args.rows, args.cols, 3), np.uint8)
    DEP = np.zeros((nf, 8, args.rows, args.cols), np.uint16)
    for j in range(nf):
        b, d = R.synth_frame_rt(args.rows, args.cols, rt8, SEED, R.synth_path_pose(SEED, p0 + j))
        BGR[j], DEP[j] = b, d
    gen_s = time.perf_counter() - t_gen
    pinned = R.HostPinned(BGR, DEP) if os.environ.get("R360_NO_PIN") != "1" else R.HostPinned()

    def frames_of(i):
        return BGR[i - p0], DEP[i - p0]

    params = R.IcpParams.default()
    params.n_pyr = 5
    params.std_dev_photo = np.float32(3.0 / 255)       # OdometryRGBD360.cpp:92-95
    params.fixed_iters_level0 = args.iters0
    runner = (runner_factory or OD.SequenceRunner)(local, args.rows, args.cols, P, params,
                                                   planes=args.workload != "dense", dense_only=args.workload == "dense",
                                                   queue=args.queue, planes_only=args.workload == "planes",
                                                   depth=args.depth, lookahead=args.lookahead,
                                                   **({"plane_batch": args.plane_batch} if runner_factory is None else {}))
    ctxs = runner.ctxs + ([runner.queue.ctx] if runner.queue else [])
    dense_ctx = runner.queue.ctx if runner.queue else ctxs[0]   # where pipeline 0's alignments run

    def barrier():
        if group is not None:
            group.barrier(ctxs)

    # warmup: every buffer (frames, queues, records) is allocated here, outside the timed region
    wrec = np.zeros((max(args.warmup, 1), p1 - p0, OD.REC), np.float32)
    runner.run(p0, p1, frames_of, wrec, repeats=max(args.warmup, 1), runs=runs)
    # frame builds per step beyond one per pair: the first frame of every segment of every piece
    halo_per_step = ((len(runs) * args.steps) if runs else
                     sum(len(g) for g in OD.stream_pieces(p0, p1, args.steps, P))) / args.steps

    rec = np.zeros((args.steps, p1 - p0, OD.REC), np.float32)
    runner.host_s[:] = 0
    if hasattr(runner, "host_detail"):
        runner.host_detail[:] = 0
    for c in runner.ctxs:
        c.host_times(reset=True)
    barrier()
    # HIP events around the level-0 passes (on the stream they are launched on); every launch only with
    # --stage-timing (events around every plane kernel of 16 streams cost throughput)
    for c in ctxs:
        c.timing(1 if args.stage_timing else 2)
        c.timing_reset()
        c.kernel_time_reset()
    q0 = runner.queue.stats() if runner.queue else None
    pq0 = runner.plane_stats() if hasattr(runner, "plane_stats") else None
    ru0 = os.times()
    th0 = thread_cpu_s()
    t0 = time.perf_counter()
    runner.run(p0, p1, frames_of, rec, repeats=args.steps, runs=runs)
    t_run = time.perf_counter() - t0
    t_g = time.perf_counter()
    if group is not None:   # RCCL gather of the pair records over xGMI
        allrec, sizes = gather_records(group.allgather, rec, -(-(args.frames - 1) // shard_world))
    else:
        allrec, sizes = rec, [p1 - p0]
    gather_s = time.perf_counter() - t_g
    traj = OD.compose(allrec[-1]) if rank == 0 else None   # OdometryRGBD360.cpp:257
    elapsed = time.perf_counter() - t0
    ru1 = os.times()
    th1 = thread_cpu_s()
    host_cores_busy = ((ru1.user - ru0.user) + (ru1.system - ru0.system)) / elapsed   # this rank's process
    pipe_s = sum(th1[t] - th0.get(t, 0.0) for t in th1 if t in runner.native_ids)
    live_s = sum(th1[t] - th0.get(t, 0.0) for t in th1 if t not in runner.native_ids)
    host_split = {"pipeline_threads": round(pipe_s / elapsed, 2), "other_live_threads": round(live_s / elapsed, 2),
                  "exited_threads": round(host_cores_busy - (pipe_s + live_s) / elapsed, 2),
                  "other_live_top": sorted((round((th1[t] - th0.get(t, 0.0)) / elapsed, 2) for t in th1
                                            if t not in runner.native_ids), reverse=True)[:6]}
    barrier()
    # interpretation-tree searches of the pipelines' RegisterPbMap calls (warm-up + timed), and how many of them stopped
    # at the node budget (r360_ctx_match_stats; none may: the search is then exhaustive, as MRPT's)
    mstats = np.sum([c.match_stats() for c in runner.ctxs], axis=0) if runner.ctxs else np.zeros(3)
    matcher = {"searches": int(mstats[0]), "budget_hits": int(mstats[1]),
               "max_nodes": int(max([c.match_stats()[2] for c in runner.ctxs] or [0]))}
    l0_ms, l0_n, k0_us, k0_n, k0_jobs, stage, coarse = 0.0, 0, 0.0, 0, 0, {}, {}
    qstats = None
    if runner.queue:   # batches of the timed run
        q1 = runner.queue.stats()
        qstats = {"batches": q1["batches"] - q0["batches"], "jobs": q1["jobs"] - q0["jobs"], "max_batch": q1["max_batch"]}
    pqstats = None
    if pq0 is not None:   # the plane queue's batches of the timed run
        pq1 = runner.plane_stats()
        pqstats = {"batches": pq1["batches"] - pq0["batches"], "frames": pq1["frames"] - pq0["frames"],
                   "max_batch": pq1["max_batch"]}
        pqstats["mean_batch"] = pqstats["frames"] / max(pqstats["batches"], 1)
    for c in ctxs:
        c.timing(False)
        ms, n = c.timing_read("k_icp_pass_L0")
        l0_ms += ms
        l0_n += n
        us, n, nj = c.kernel_stats(0)
        k0_us += us
        k0_n += n
        k0_jobs += nj
        for lv in range(1, 5):   # the coarse levels (diagnostic): launches that ran a job, their in-kernel span
            us, n, nj = c.kernel_stats(lv)
            kc = coarse.setdefault(lv, [0.0, 0, 0])
            kc[0] += us
            kc[1] += n
            kc[2] += nj
        for name in ("k_undistort", "k_stitch", "k_pyramid", "k_cloud", "k_bilateral", "k_distmap", "k_normals",
                     "k_ccl", "k_plane_fit", "k_refine", "k_model_stats", "k_icp_pass", "k_icp_pass_L0"):
            ms, n = c.timing_read(name)
            stage[name] = stage.get(name, 0.0) + ms
    hs = runner.host_s.sum(axis=0)
    host_ms = {k: 1e3 * v / max(hs[3], 1) for k, v in zip(("load_build_enqueue", "pbmap_stage", "dense_wait"), hs[:3])}
    if hasattr(runner, "host_detail"):   # inside load_build_enqueue
        hd = runner.host_detail.sum(axis=0)
        host_ms["load_split"] = {k: 1e3 * v / max(hs[3], 1) for k, v in
                                 zip(("build_enqueue", "upload_enqueue", "refill_collects", "edge_waits"), hd)}
    ht = np.sum([c.host_times() for c in runner.ctxs], axis=0)   # inside RegisterPbMap
    host_ms["pbmap_stage_split"] = {k: 1e3 * v / max(ht[3], 1) for k, v in
                                    zip(("wait_frame_pbmaps", "match_tables", "tree_and_pose"), ht[:3])}
    host_ms["pbmap_assembly_per_frame"] = 1e3 * ht[4] / max(ht[5], 1)
    per_rank = None
    if group is not None:
        # per-rank figures for diagnosing a scaling run from its own line: pairs, time to the end of its shard, the
        # record gather's share of the timed region, and the halo frames (one per pipeline run) it rebuilt
        mine = np.array([rank, p1 - p0, elapsed, t_run, gather_s, halo_per_step, P], np.float64)
        allm = group.allgather(mine.astype(np.float32))
        per_rank = [{"rank": int(m[0]), "pairs_per_step": int(m[1]), "pairs_per_s": float(m[1] * args.steps / m[2]),
                     "shard_s": float(m[3]), "timed_s": float(m[2]), "gather_ms": float(m[4] * 1e3),
                     "halo_frames_per_step": float(m[5]), "pipelines": int(m[6])} for m in allm]
        elapsed = group.max(elapsed)
    pairs_job = args.steps * sum(sizes)
    value = pairs_job / elapsed
    # every timed step's pair records against the first warm-up step's, bit for bit (the same pairs, registered in
    # other pipeline pieces and dense batches): a wrong frame buffer at a piece's repeat boundary would show here
    records_same = {"timed_steps": bool((rec == wrec[0][None]).all()),
                    "warmup_steps": bool((wrec == wrec[0][None]).all())}

    # secondary: the same steps with the raw images already resident in HBM (device-to-device copies
    # into the frames instead of PCIe uploads)
    resident = None
    if not args.no_resident:
        dB, dD = R.DeviceArray(local, BGR), R.DeviceArray(local, DEP)

        def dev_of(i):
            return dB.ptr(i - p0), dD.ptr(i - p0)
        rec2 = np.zeros((args.steps, p1 - p0, OD.REC), np.float32)
        for c in ctxs:
            c.timing(1 if args.stage_timing else 2)   # same event instrumentation as the headline run
        barrier()
        t1 = time.perf_counter()
        runner.run(p0, p1, dev_of, rec2, repeats=args.steps, runs=runs, device_inputs=True)
        e2 = time.perf_counter() - t1
        for c in ctxs:
            c.timing(False)
            c.timing_reset()
        if group is not None:
            e2 = group.max(e2)
        resident = pairs_job / e2
        dB.close()
        dD.close()
        records_same["resident_steps"] = bool((rec2 == wrec[0][None]).all())

    W0 = args.rows * 8
    H0 = int(W0 * 0.5 * 60.0 / 180)               # Frame360.h:391-392 (640 x 3840 at VGA)
    N0 = H0 * W0
    sso = float(np.mean(rec[:, :, OD.R_SSO]))
    V = sso * N0
    alg_bytes = 8.0 * N0 + 24.0 * V               # B = 8 N + 24 V per pass
    # The pass's duration is its in-kernel execution span (earliest workgroup start to the end of the
    # last workgroup, s_memrealtime), which is what rocprofv3's kernel trace reports; stream events
    # around a launch also count the time it waits behind the other pipelines' kernels.
    avg_ms = k0_us / max(k0_n, 1) * 1e-3
    event_ms = l0_ms / max(l0_n, 1)
    pairs_per_launch = k0_jobs / max(k0_n, 1)      # a batched launch runs one level-0 pass per pair
    achieved = pairs_per_launch * alg_bytes / (avg_ms * 1e-3) / 1e9 if k0_n else None
    # a lone pair on an idle GPU (OdometryRGBD360's sequential caller registers one pair at a time): the sequence's
    # first two frames built through the façade, alignFrames360 with the same schedule, nothing else running
    iso_ms, n, iso_ach, lone_ms, lone_mean_ms = 0.0, 0, None, None, None
    if not args.no_isolated:
        # two consecutive frames of the sequence, built as a caller of the façade builds them, on a context of their
        # own (the runner's queued ring frames skip the compacted level-0 points a lone pass reads)
        ictx = R.Context(local)
        ical = R.Calib360(ictx, args.rows, args.cols)
        ical.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
        fa, fb = R.Frame360(ical), R.Frame360(ical)
        for f, j in ((fa, p0), (fb, p0 + 1)):
            f.upload(*frames_of(j))
            f.build()
        reg = R.RegisterPhotoICP(ictx)
        reg.params = params
        reg.setTargetFrame(fa)
        reg.setSourceFrame(fb)
        for _ in range(2):
            reg.alignFrames360(np.eye(4, dtype=np.float32), R.PHOTO_DEPTH)
        ictx.sync()
        ictx.kernel_time_reset()
        tl = []
        for _ in range(20):   # median of 20 (one late host wake-up would move a 5-call mean by ~2 %)
            t_l = time.perf_counter()
            reg.alignFrames360(np.eye(4, dtype=np.float32), R.PHOTO_DEPTH)
            tl.append(time.perf_counter() - t_l)
        lone_ms = float(np.median(tl)) * 1e3
        lone_mean_ms = float(np.mean(tl)) * 1e3
        us, n, nj = ictx.kernel_stats(0)
        iso_ms = us / max(n, 1) * 1e-3
        iso_ach = (nj / max(n, 1)) * alg_bytes / (iso_ms * 1e-3) / 1e9 if n else None
        del reg, fa, fb, ical, ictx   # the frames and calibration hold their context: it goes last
    probe = None
    if args.eval_probe:   # opt-in diagnostic: the level-0 pass in eval mode (no GN step) at identity, alone
        fa, fb = runner.frames[0][:2]
        reg = R.RegisterPhotoICP(ctxs[0])
        reg.setNumPyr(5)
        reg.setGrayVariance(3.0 / 255)
        reg.setTargetFrame(fa)
        reg.setSourceFrame(fb)
        for _ in range(3):
            reg.eval(0, np.eye(4, dtype=np.float32), R.PHOTO_DEPTH)
        ctxs[0].kernel_time_reset()
        for _ in range(30):
            reg.eval(0, np.eye(4, dtype=np.float32), R.PHOTO_DEPTH)
        ctxs[0].sync()
        pu, pn = ctxs[0].kernel_time(0)
        probe = {"avg_launch_ms": pu / max(pn, 1) * 1e-3, "launches": pn,
                 "note": "eval mode at identity pose, pipeline 0's last pair, in-kernel span"}
    # HBM bytes per level-0 launch from the rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes of this same
    # command (tools/profile.sh + tools/profile_summary.py, committed under profiles/); reported only when
    # the profile measured the current ICP sources
    traffic, traffic_src = None, None
    tf = os.path.join(ROOT, "profiles", "latest", "l0_pass.json")
    if os.path.exists(tf) and (args.rows, args.cols, args.workload) == (480, 640, "sequence"):
        prof = json.load(open(tf))
        if prof.get("icp_source_hash") == icp_source_hash() and prof.get("hbm_bytes_per_pair_pass"):
            # the profile's HBM bytes per pair-pass, scaled to this run's pairs per launch
            traffic, traffic_src = prof["hbm_bytes_per_pair_pass"] * pairs_per_launch, prof.get("tag")
    steps_pairs = p1 - p0
    if args.workload == "sequence":
        workload = ("config4 (per pair configs 1+2's work): OdometryRGBD360 over the synthetic "
                    f"{args.frames}-frame sequence, 8x{args.cols}x{args.rows}; each step registers every "
                    "consecutive pair once: upload of the new frame's raw images, Frame360 build on the GPU "
                    "(undistort, cloud + median downsample, bilateral, normals, plane segmentation + "
                    "refinement, PbMap descriptors/grouping, stitch, 5-level pyramid), RegisterPbMap(25 planes, "
                    "PLANAR_3DoF) + alignFrames360(PHOTO_DEPTH) from the rotOffset-conjugated PbMap pose "
                    f"(levels 4..1 reference schedule + {args.iters0} GN iterations at level 0), pose gather + "
                    "trajectory composition on rank 0")
    elif args.workload == "planes":
        workload = ("config2 over the config4 sequence: per pair upload + Frame360 build with planes (PbMap) + "
                    "RegisterPbMap(25 planes, PLANAR_3DoF), no alignFrames360")
    else:
        workload = (("config5" if args.rows == 960 else "config3") + f": synthetic 8x{args.cols}x{args.rows} "
                    f"{args.frames}-frame sequence; per pair: upload, stitch + 5-level pyramid, "
                    f"alignFrames360(PHOTO_DEPTH) levels 4..1 reference schedule + {args.iters0} GN iterations "
                    "at level 0")
    out = {
        "metric": METRIC, "value": value, "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {
            "workload": workload, "sensors": f"8x{args.cols}x{args.rows}", "sphere": f"{H0}x{W0}",
            "n_pyr": 5, "parallelism": f"pair-shard dp{world}", "pairs_per_step": pairs_job // args.steps,
            "pairs_per_step_this_rank": steps_pairs, "pipelines_per_gpu": P,
            "pipeline_work": ("one run of each step per pipeline" if runs else
                              "the steps x pairs stream cut into one contiguous piece per pipeline"),
            "extra_frame_builds_per_step": halo_per_step,
            "dense_batch": args.queue, "dense_in_flight_per_pipeline": args.depth if args.queue else 1,
            "frames_built_ahead": args.lookahead if args.queue else 1,
            "plane_batch": args.plane_batch,
            # the hardware-queue pool this run had (bench.py sets 16 only where the environment left it unset)
            "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            # the library the binding loaded (R360_LIB can point the binding elsewhere: shown, never silent)
            "library": os.path.relpath(R.LIB_PATH, ROOT), "library_sha16": _sha16(R.LIB_PATH),
            **({"emulated_shard": f"{shard_rank}/{shard_world}"} if args.emulate else {}),
        },
        "value_hbm_resident_inputs": resident,
        "records_identical": all(records_same.values()),
        "records_check": {**records_same, "reference": "first warm-up step, same runner mode",
                          **({"ranks": "per rank, own shard"} if group is not None else {})},
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
            "traffic_profile": traffic_src,
            "traffic_per_pair_pass": (traffic / pairs_per_launch) if traffic else None,
            "kernel": "k_icp_pass<PHOTO_DEPTH> (level 0)", "avg_launch_ms": avg_ms, "launches": k0_n,
            "pairs_per_launch": pairs_per_launch,
            "timing": "in-kernel execution span (s_memrealtime) over the timed region, all pipelines running",
            "event_avg_launch_ms": event_ms, "bytes_per_launch": pairs_per_launch * alg_bytes,
            "bytes_per_pair_pass": alg_bytes, "visible_frac": sso,
            "isolated": {"avg_launch_ms": iso_ms, "launches": n, "achieved": iso_ach,
                         "frac": (iso_ach / HBM_PEAK_GBS) if iso_ach else None, "align_ms_per_pair": lone_ms, "align_ms_per_pair_mean": lone_mean_ms,
                         "note": "a lone pair on an idle GPU: alignFrames360 (same schedule) of two built frames, "
                                 "one pair per launch, 5 calls after 2 warm-up calls"},
            **({"eval_probe": probe} if probe else {}),
        },
        **({"stage_ms_per_pair": {k: v / max(args.steps * steps_pairs, 1) for k, v in stage.items()}}
           if args.stage_timing else {}),
        "coarse_levels": {f"L{lv}": {"launches": v[1], "avg_launch_us": v[0] / max(v[1], 1), "pair_passes": v[2],
                                     "ms_per_step": v[0] * 1e-3 / args.steps} for lv, v in sorted(coarse.items())},
        "pipeline_host_ms_per_pair": host_ms,
        "pbmap_matcher": matcher, "pbmap_budget_hits": matcher["budget_hits"],
        "runner": "C++ (r360_sequence, rgbd360_amd/csrc/host/sequence.cpp)",
        "host_cores_busy": round(host_cores_busy, 2),
        "host_cores_split": host_split,
        **({"dense_queue": {**qstats, "mean_batch": qstats["jobs"] / max(qstats["batches"], 1)}} if qstats else {}),
        **({"plane_queue": pqstats} if pqstats and pqstats["batches"] else {}),
        **({"per_rank": per_rank} if per_rank else {"gather_ms": gather_s * 1e3}),
        "frame_generation_s": round(gen_s, 1),
    }
    if rank == 0 and traj is not None:
        gt = np.stack([R.synth_path_pose(SEED, k).astype(np.float64) for k in range(args.frames)])
        if allrec.shape[1] == args.frames - 1:
            out["trajectory"] = OD.trajectory_error(traj, gt)
            st = allrec[-1, :, OD.R_STATUS]
            out["trajectory"].update({"pairs": int(allrec.shape[1]), "pbmap_failed": int((st == 1).sum()),
                                      "illposed": int((st == 2).sum())})
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(runner.cals[0], frames_of, p0, p1, args.workload, args.iters0)
    runner.close()
    if rank == 0 and world == 1 and not args.no_halves and args.workload == "sequence":
        out["sequential_cpp"] = sequential_leg(local, args.rows, args.cols, p0, frames_of, params)
        out["config1"] = config1_leg(local)
    # configs[1] and configs[2] (the two halves of each pair's work) over the same sequence, after the timed region
    if rank == 0 and world == 1 and not args.no_halves and args.workload == "sequence":
        out["config2"] = half_leg("planes", local, args.rows, args.cols, p0, p1, frames_of, params, args.streams,
                                  args.queue, args.depth)
        out["config3"] = half_leg("dense", local, args.rows, args.cols, p0, p1, frames_of, params, args.streams,
                                  args.queue, args.depth)
    pinned.close()
    if rank == 0 and world == 1 and not args.no_config5 and args.workload == "sequence" and args.rows == 480:
        del BGR, DEP
        out["config5"] = config5_leg(local, rt8)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if group is not None:
        group.close()


if __name__ == "__main__":
    main()
