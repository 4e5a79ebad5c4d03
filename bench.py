"""bench.py — registered Frame360 pairs/sec on MI355X (BASELINE.json metric) + ICP-reduce roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload full|dense]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload "full" (default; BASELINE.json configs[1]+[2] as one registration, run the way configs[3]
runs them): the synthetic 256-frame OdometryRGBD360 sequence (procedural room, seed 360, 8 x 480x640
sensors).  One step registers, on each of P pipelines of each GPU, the next consecutive pair of the
rank's shard (pipelines run free on their own host threads and HIP streams; the timed region covers
`steps` pairs per pipeline): the new Frame360 is built end to end on the GPU (undistort, cloud + 2x2 median
downsample, bilateral filter, normals, plane segmentation + refinement, PbMap descriptors and
grouping, spherical stitch, 5-level pyramid with gradients), then RegisterRGBD360::RegisterPbMap
(25 planes, PLANAR_3DoF) and RegisterPhotoICP::alignFrames360(PHOTO_DEPTH) initialised with the
rotOffset-conjugated PbMap pose (OdometryKeyFrame360.cpp:205-254), with the reference schedule on
levels 4..1 and exactly 20 Gauss-Newton iterations at level 0 (timing mode).
Workload "dense" (configs[2] alone): stitch + pyramid of both frames + alignFrames360.
Raw sensor images are resident in HBM before the timed region.  Multi-GPU: each rank registers its
own contiguous shard of the sequence (weak scaling, no data-path collective) and the 4x4 poses are
gathered with one RCCL all_gather over xGMI.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# Hardware queues per process (HIP's default is 4): the per-frame plane kernels are latency-bound
# (one workgroup or wave per sensor), so throughput comes from many pipelines' kernels running at
# once; 16 queues let 16+ streams reach the hardware side by side.  Must precede HIP initialisation.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

METRIC = "registered Frame360 pairs/sec @ 8×640×480; ICP-reduce HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
SEQ_LEN = 256


def shard_windows(rank, world, pipelines, window, seq_len=SEQ_LEN):
    """Frame indices each pipeline of this rank walks: the rank owns a contiguous shard of the sequence
    (pairs are independent); pipeline p takes a window of `window` consecutive frames in it."""
    shard = seq_len // world
    first = rank * shard
    span = max(1, shard - window)
    return [list(range(first + (p * window) % span, first + (p * window) % span + window)) for p in range(pipelines)]


def gather_poses(dist, poses, device):
    """One all_gather of every rank's poses (RCCL over xGMI with backend nccl; gloo on CPU in the tests)."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(poses, np.float32).reshape(-1, 16)).to(device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return torch.cat(out).cpu().numpy()


def max_over_ranks(dist, value, device):
    import torch
    e = torch.tensor([value], device=device, dtype=torch.float64)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return float(e.item())


def cpu_baseline(R, cal, seed, first, workload, iters0, budget_s=15.0):
    """The CPU oracle (C++ restatement, OpenMP over the 8 sensors / rows) on a bounded sample of the
    same workload: consecutive pairs of the same synthetic sequence."""
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

    def frame(i):
        b, d = cal.synth_frame(seed, R.synth_path_pose(seed, i))
        return b, d

    def build(b, d):
        sb, sd = O.stitch(b, d, rti, Km)
        pm = O.PbMap(d.astype(np.float32) * np.float32(0.001), b, rt8) if workload == "full" else None
        return sb, sd, pm

    raw = [frame(first + j) for j in range(6)]
    prev = build(*raw[0])
    n, t0 = 0, time.perf_counter()
    while True:
        b, d = raw[(n + 1) % len(raw)]
        cur = build(b, d)
        if workload == "full":
            r = O.register_pbmap(prev[2], cur[2], 25, O.PLANAR_3DoF)
            init = Ro @ (r["pose"] if r["good"] else np.eye(4, dtype=np.float32)) @ Ri
        else:
            prev = build(*raw[n % len(raw)])     # dense: both frames per pair
            init = None
        O.align360(prev[0], prev[1], cur[0], cur[1], init, O.PHOTO_DEPTH, prm)
        prev = cur
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    what = ("PbMap build of the new frame + RegisterPbMap + stitch + alignFrames360" if workload == "full"
            else "stitch x2 + alignFrames360")
    return {"value": n / dt, "unit": "pairs/s", "cores": cores, "kind": "port",
            "sample": f"{n} consecutive synthetic 8x480x640 pairs ({what}, nPyr=5, {iters0} level-0 iterations), "
                      f"oracle/liboracle360.so, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=480)
    ap.add_argument("--cols", type=int, default=640)
    ap.add_argument("--iters0", type=int, default=20)
    ap.add_argument("--workload", choices=["full", "dense"], default="full")
    ap.add_argument("--streams", type=int, default=16, help="pairs in flight per GPU (one pipeline = host thread + HIP stream each)")
    ap.add_argument("--window", type=int, default=16, help="sequence frames resident per pipeline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eval-probe", action="store_true", help="diagnostic: also time the level-0 pass in eval mode")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    import rgbd360_amd as R

    # P independent pipelines (one r360_ctx = one HIP stream + device GN state each) keep several pairs
    # in flight: one pipeline's host-side PbMap work and latency-bound coarse ICP levels overlap the
    # other pipelines' kernels
    P = max(1, args.streams)
    F = max(3, args.window)
    ctxs = [R.Context(local) for _ in range(P)]
    cals = []
    for c in ctxs:
        cal = R.Calib360(c, args.rows, args.cols)
        cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
        cals.append(cal)
    cal = cals[0]
    seed = 360 << 16
    # this rank's shard of the 256-frame sequence; pipeline p walks its own contiguous window of it
    windows = shard_windows(rank, world, P, F)
    first = windows[0][0]
    flags = R.BUILD_UNDISTORT | R.BUILD_SPHERE | R.BUILD_PYRAMID
    if args.workload == "full":
        flags |= R.BUILD_PLANES
    frames = []
    raw = {}
    for p, c in enumerate(cals):
        fl = []
        for idx in windows[p]:
            if idx not in raw:
                raw[idx] = cal.synth_frame(seed, R.synth_path_pose(seed, idx))
            b, d = raw[idx]
            f = R.Frame360(c)
            f.upload(b, d)          # raw 8-sensor images resident in HBM before timing
            f.build(flags)          # allocates every device buffer outside the timed region
            fl.append(f)
        frames.append(fl)
    params = R.IcpParams.default()
    params.n_pyr = 5
    params.std_dev_photo = np.float32(3.0 / 255)       # OdometryRGBD360.cpp:92-95
    params.fixed_iters_level0 = args.iters0
    L = R.lib()
    eye16 = np.eye(4, dtype=np.float32).reshape(16)
    pout = np.zeros((P, 16), np.float32)
    stats = [R.IcpStats() for _ in range(P)]

    prof = os.environ.get("BENCH_PROFILE") is not None
    tacc = np.zeros((P, 4))

    def pair(p, k, out):
        """Pipeline p registers its k-th pair (frames j, j+1 of its window) and writes the pose to out."""
        ta = time.perf_counter()
        j = k % (F - 1)
        if args.workload == "dense" or j == 0:
            frames[p][j].build(flags, sync=False)
        frames[p][j + 1].build(flags, sync=False)
        ref, trg = frames[p][j], frames[p][j + 1]
        tb = time.perf_counter()
        if args.workload == "full":   # PbMap stage on this host thread, then the dense stage is enqueued
            rc = L.r360_register_async(ctxs[p].h, ref.h, trg.h, R._fptr(eye16), R.C.byref(params), 25,
                                       R.PLANAR_3DoF)
        else:
            rc = L.r360_align360_async(ctxs[p].h, ref.h, trg.h, R._fptr(eye16), R.PHOTO_DEPTH, 0,
                                       R.C.byref(params))
        assert rc == 0, L.r360_last_error()
        tc = time.perf_counter()
        if args.workload == "full":
            rc = L.r360_register_result(ctxs[p].h, R._fptr(out), None, R.C.byref(stats[p]))
        else:
            rc = L.r360_align360_result(ctxs[p].h, R._fptr(out), None, None, R.C.byref(stats[p]))
        assert rc >= 0, L.r360_last_error()
        if prof:
            tacc[p] += (tb - ta, tc - tb, time.perf_counter() - tc, 1)

    # Each pipeline runs free on its own host thread (ctypes drops the GIL inside the library), so one
    # pipeline's host PbMap stage and its wait for results never stall the others' GPU work.
    pool = ThreadPoolExecutor(max_workers=P)

    def run(k0, n, poses):
        def worker(p):
            for i in range(n):
                pair(p, k0 + i, poses[i, p])
        for f in [pool.submit(worker, p) for p in range(P)]:
            f.result()

    run(0, args.warmup, np.zeros((max(args.warmup, 1), P, 16), np.float32))
    for c in ctxs:
        c.sync()

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    poses = np.zeros((args.steps, P, 16), np.float32)
    barrier()
    for c in ctxs:
        c.timing(True)
        c.timing_reset()
        c.kernel_time_reset()
    t0 = time.perf_counter()
    run(args.warmup, args.steps, poses)
    for c in ctxs:
        c.sync()
    if dist is not None:  # RCCL pose gather over xGMI
        import torch
        gather_poses(dist, poses, "cuda")
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if prof:
        n = max(tacc[:, 3].sum(), 1)
        print(f"per pair (ms): build-enqueue {1e3 * tacc[:, 0].sum() / n:.2f}  pbmap-stage {1e3 * tacc[:, 1].sum() / n:.2f}"
              f"  dense-wait {1e3 * tacc[:, 2].sum() / n:.2f}", file=sys.stderr)
    barrier()
    l0_ms, l0_n = 0.0, 0        # stream events around each level-0 pass
    k0_us, k0_n = 0.0, 0        # in-kernel execution spans of the same passes
    stage = {}
    for c in ctxs:
        c.timing(False)
        ms, n = c.timing_read("k_icp_pass_L0")
        l0_ms += ms
        l0_n += n
        us, n = c.kernel_time(0)
        k0_us += us
        k0_n += n
        for name in ("k_cloud", "k_bilateral", "k_distmap", "k_normals", "k_ccl", "k_plane_fit", "k_refine",
                     "k_model_stats", "k_icp_pass", "k_icp_pass_L0"):
            ms, n = c.timing_read(name)
            stage[name] = stage.get(name, 0.0) + ms
    if dist is not None:
        elapsed = max_over_ranks(dist, elapsed, "cuda")

    total_pairs = args.steps * world * P
    value = total_pairs / elapsed
    W0 = args.rows * 8
    H0 = int(W0 * 0.5 * 60.0 / 180)               # Frame360.h:391-392 (640 x 3840 at VGA)
    N0 = H0 * W0
    sso = float(stats[0].sso)
    V = sso * N0
    alg_bytes = 8.0 * N0 + 24.0 * V            # B = 8 N + 24 V per pass
    # The pass's duration is its in-kernel execution span (earliest workgroup start to the end of the
    # last workgroup, s_memrealtime), which is what rocprofv3's kernel trace reports; stream events
    # around a launch also count the time it waits behind the other pipelines' kernels.
    avg_ms = k0_us / max(k0_n, 1) * 1e-3
    event_ms = l0_ms / max(l0_n, 1)
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9 if k0_n else None
    # the same pass with the GPU to itself: pipeline 0 registers a few more pairs alone
    for c in ctxs:
        c.kernel_time_reset()
    iso = np.zeros((3, P, 16), np.float32)
    for i in range(3):
        pair(0, args.warmup + args.steps + i, iso[i, 0])
    ctxs[0].sync()
    us, n = ctxs[0].kernel_time(0)
    iso_ms = us / max(n, 1) * 1e-3
    iso_ach = alg_bytes / (iso_ms * 1e-3) / 1e9 if n else None
    probe = None
    if args.eval_probe:   # opt-in diagnostic: the level-0 pass in eval mode (no GN step) at identity, alone
        j = (args.warmup + args.steps + 2) % (F - 1)
        reg = R.RegisterPhotoICP(ctxs[0])
        reg.setNumPyr(5); reg.setGrayVariance(3.0 / 255)
        reg.setTargetFrame(frames[0][j]); reg.setSourceFrame(frames[0][j + 1])
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
    # command (tools/profile.sh + tools/profile_summary.py, committed under profiles/)
    traffic = None
    tf = os.path.join(ROOT, "profiles", "latest", "l0_pass.json")
    if os.path.exists(tf) and (args.rows, args.cols, args.workload) == (480, 640, "full"):
        traffic = json.load(open(tf)).get("hbm_bytes_per_launch")   # profiled on the default workload only
    pairs_timed = args.steps * P
    if args.workload == "full":
        workload = ("config2+3 (run as config4's sequence): per pair, the new synthetic "
                    f"8x{args.cols}x{args.rows} Frame360 is "
                    "built on the GPU (undistort, cloud + median downsample, bilateral, normals, plane "
                    "segmentation + refinement, PbMap descriptors/grouping, stitch, 5-level pyramid), then "
                    "RegisterPbMap(25 planes, PLANAR_3DoF) + alignFrames360(PHOTO_DEPTH) initialised with the "
                    f"rotOffset-conjugated PbMap pose: levels 4..1 reference schedule + {args.iters0} GN "
                    "iterations at level 0")
    else:
        workload = (("config5" if args.rows == 960 else "config3") + f": synthetic 8x{args.cols}x{args.rows} "
                    "Frame360 pair -> stitch + 5-level pyramid x2 -> "
                    f"alignFrames360(PHOTO_DEPTH) levels 4..1 reference schedule + {args.iters0} GN iterations "
                    "at level 0")
    out = {
        "metric": METRIC, "value": value, "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {
            "workload": workload, "sensors": f"8x{args.cols}x{args.rows}", "sphere": f"{H0}x{W0}",
            "n_pyr": 5, "parallelism": f"pair-per-GPU dp{world}", "pairs_in_flight_per_gpu": P,
            "pairs_per_step_per_gpu": P,
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
            "kernel": "k_icp_pass<PHOTO_DEPTH> (level 0)", "avg_launch_ms": avg_ms, "launches": k0_n,
            "timing": "in-kernel execution span (s_memrealtime) over the timed region, all pipelines running",
            "event_avg_launch_ms": event_ms, "bytes_per_launch": alg_bytes, "visible_frac": sso,
            "isolated": {"avg_launch_ms": iso_ms, "launches": n, "achieved": iso_ach,
                         "frac": (iso_ach / HBM_PEAK_GBS) if iso_ach else None,
                         "note": "same pass, pipeline 0 alone on the GPU (3 pairs after the timed region)"},
            **({"eval_probe": probe} if probe else {}),
        },
        "stage_ms_per_pair": {k: v / max(pairs_timed, 1) for k, v in stage.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(R, cal, seed, first, args.workload, args.iters0)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
