"""bench.py — registered Frame360 pairs/sec on MI355X (BASELINE.json metric) + ICP-reduce roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2], "single synthetic 8x640x480 pair, full RegisterPhotoICP (20 iters)
with JtJ reduction"): one step = one Frame360 pair of the synthetic 256-frame sequence (procedural
room, seed 360) registered end to end on the GPU — both frames stitched (8 x 480x640 -> 640x3840
sphere) and pyramided (5 levels, gray + depth + target gradients), then
RegisterPhotoICP::alignFrames360(PHOTO_DEPTH) with the reference schedule on levels 4..1 and exactly
20 Gauss-Newton iterations at level 0 (timing mode).  Raw sensor images are resident
in HBM before the timed region.  Multi-GPU: pair-per-GPU sharding of the sequence (weak scaling,
no data-path collective) + one RCCL all_gather of the resulting 4x4 poses.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "registered Frame360 pairs/sec @ 8×640×480; ICP-reduce HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md


def make_pair_frames(R, cal, seed, i):
    A = R.synth_path_pose(seed, i)
    B = R.synth_path_pose(seed, i + 1)
    return cal.synth_frame(seed, A), cal.synth_frame(seed, B)


def cpu_baseline(R, cal, pairs, fixed_iters, budget_s=12.0):
    """The CPU oracle (C++ restatement, OpenMP) on a bounded sample of the same workload."""
    from oracle import oracle360 as O
    _, rti, K = cal.extrinsics()
    Km = K.reshape(3, 3).T
    prm = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255), fixed_iters_level0=fixed_iters)
    n, t0 = 0, time.perf_counter()
    while True:
        (b1, d1), (b2, d2) = pairs[n % len(pairs)]
        s1b, s1d = O.stitch(b1, d1, rti, Km)
        s2b, s2d = O.stitch(b2, d2, rti, Km)
        O.align360(s1b, s1d, s2b, s2d, None, O.PHOTO_DEPTH, prm)
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": n / dt, "unit": "pairs/s", "cores": cores, "kind": "port",
            "sample": f"{n} synthetic 8x480x640 pairs (cycling {len(pairs)}) (stitch x2 + alignFrames360 nPyr=5, "
                      f"{fixed_iters} level-0 iterations), oracle/liboracle360.so, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=480)
    ap.add_argument("--cols", type=int, default=640)
    ap.add_argument("--iters0", type=int, default=20)
    ap.add_argument("--streams", type=int, default=8, help="pairs in flight per GPU (one HIP stream each)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
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
    # in flight, so the latency-bound coarse pyramid levels of one pair overlap other pairs' work
    P = max(1, args.streams)
    ctxs = [R.Context(local) for _ in range(P)]
    cals = []
    for c in ctxs:
        cal = R.Calib360(c, args.rows, args.cols)
        cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
        cals.append(cal)
    cal = cals[0]
    seed = 360 << 16

    # this rank's shard of the 256-frame sequence: consecutive pairs, one pair per pipeline per step
    n_frames_local = 4
    first = (rank * 32) % 252
    raw = [cal.synth_frame(seed, R.synth_path_pose(seed, first + j)) for j in range(n_frames_local)]
    frames = []
    for c in cals:
        fl = []
        for (b, d) in raw:
            f = R.Frame360(c)
            f.upload(b, d)  # raw 8-sensor images resident in HBM before timing
            fl.append(f)
        frames.append(fl)
    regs = []
    for c in ctxs:
        reg = R.RegisterPhotoICP(c)
        reg.setNumPyr(5)
        reg.setGrayVariance(3.0 / 255)
        reg.params.fixed_iters_level0 = args.iters0
        regs.append(reg)
    L = R.lib()
    init16 = np.eye(4, dtype=np.float32).reshape(16)
    pout = np.zeros((P, 16), np.float32)

    def step(k):
        i = k % (n_frames_local - 1)
        for p in range(P):   # enqueue every pipeline's pair, then collect
            trg, src = frames[p][i], frames[p][i + 1]
            trg.build(R.BUILD_SPHERE | R.BUILD_PYRAMID, sync=False)
            src.build(R.BUILD_SPHERE | R.BUILD_PYRAMID, sync=False)
            rc = L.r360_align360_async(ctxs[p].h, trg.h, src.h, R._fptr(init16), R.PHOTO_DEPTH, 0,
                                       R.C.byref(regs[p].params))
            assert rc == 0, L.r360_last_error()
        for p in range(P):
            rc = L.r360_align360_result(ctxs[p].h, R._fptr(pout[p]), None, None, R.C.byref(regs[p].stats))
            assert rc >= 0, L.r360_last_error()
        return pout

    for k in range(args.warmup):
        step(k)
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
    t0 = time.perf_counter()
    for k in range(args.steps):
        poses[k] = step(k)
    for c in ctxs:
        c.sync()
    if dist is not None:  # RCCL pose gather over xGMI
        import torch
        t = torch.from_numpy(poses.reshape(-1, 16)).cuda()
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    barrier()
    l0_ms, l0_n = 0.0, 0
    for c in ctxs:
        c.timing(False)
        ms, n = c.timing_read("k_icp_pass_L0")
        l0_ms += ms; l0_n += n
    reg = regs[0]
    if dist is not None:
        import torch
        e = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    total_pairs = args.steps * world * P
    value = total_pairs / elapsed
    W0 = args.rows * 8
    H0 = int(W0 * 0.5 * 60.0 / 180)               # Frame360.h:391-392 (640 x 3840 at VGA)
    N0 = H0 * W0
    sso = float(reg.stats.sso)
    V = sso * N0
    alg_bytes = 8.0 * N0 + 24.0 * V            # B = 8 N + 24 V per pass
    avg_ms = l0_ms / max(l0_n, 1)
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9 if l0_n else None
    # HBM bytes per level-0 launch from the rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes of this same
    # command (tools/profile.sh + tools/profile_summary.py, committed under profiles/)
    traffic = None
    tf = os.path.join(ROOT, "profiles", "latest", "l0_pass.json")
    if os.path.exists(tf):
        traffic = json.load(open(tf)).get("hbm_bytes_per_launch")
    out = {
        "metric": METRIC, "value": value, "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,  # one step = P pairs per GPU "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {
            "workload": "config3: synthetic 8x640x480 Frame360 pair -> stitch + 5-level pyramid x2 -> "
                        "alignFrames360(PHOTO_DEPTH) levels 4..1 reference schedule + "
                        f"{args.iters0} GN iterations at level 0",
            "sensors": f"8x{args.cols}x{args.rows}", "sphere": f"{H0}x{W0}",
            "n_pyr": 5, "parallelism": f"pair-per-GPU dp{world}", "pairs_in_flight_per_gpu": P,
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
            "kernel": "k_icp_pass<PHOTO_DEPTH> (level 0)", "avg_launch_ms": avg_ms, "launches": l0_n,
            "bytes_per_launch": alg_bytes, "visible_frac": sso,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        pairs = [make_pair_frames(R, cal, seed, first + j) for j in range(2)]
        out["cpu_baseline"] = cpu_baseline(R, cal, pairs, args.iters0)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
