"""Throughput of the batched registrations (§8f-4) against the same calls made one after another.

  python tools/bench_batch.py [--frames 24] [--lanes 8] [--reps 3]

Frames: the synthetic 8 x 480x640 sequence along the bench's camera path, built (planes, sphere, 5-level
pyramid) before timing.  Workloads, each timed sequentially (one RegisterRGBD360 / RegisterPhotoICP on one
ctx, the reference's pattern) and batched (one Batch call per frame):
  * track:  SphereGraphSLAM tracking, RegisterPbMap(PLANAR_ODOMETRY_3DoF) of each frame against its 5 newest
            predecessors (all candidates evaluated; SphereGraphSLAM.cpp:175-231)
  * lc:     LoopClosure360 checks, RegisterPbMap(PLANAR_3DoF) + gate + alignFrames360 of each frame against
            5 older keyframes (LoopClosure360.h:291-313); also all frames' candidates in one call
Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rgbd360_amd as R  # noqa: E402


def rot_offset():
    """rotOffset (OdometryRGBD360.cpp:138-139) and its inverse"""
    a = np.float64(np.float32(157.5)) * 3.14159265359 / 180
    Ro = np.eye(4, dtype=np.float32)
    c, s = np.float32(np.cos(a)), np.float32(np.sin(a))
    Ro[1, 1] = Ro[2, 2] = c
    Ro[1, 2], Ro[2, 1] = s, -s
    return Ro, Ro.T.copy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--lanes", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    seed = 360 << 16
    ctx = R.Context(0)
    cal = R.Calib360(ctx, 480, 640)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    F = []
    for i in range(a.frames):
        b, d = cal.synth_frame(seed, R.synth_path_pose(seed, i))
        f = R.Frame360(cal)
        f.upload(b, d)
        f.build(R.BUILD_UNDISTORT | R.BUILD_SPHERE | R.BUILD_PYRAMID | R.BUILD_CLOUD | R.BUILD_PLANES)
        F.append(f)
    ctx.sync()
    p = R.IcpParams.default()
    p.n_pyr = 5
    p.std_dev_photo = np.float32(3.0 / 255)
    batch = R.Batch(0, a.lanes)
    Ro, Ri = rot_offset()
    track_pairs = [(F[j], F[i]) for i in range(5, a.frames) for j in range(i - 1, i - 6, -1)]
    lc_pairs = [(F[j], F[i]) for i in range(10, a.frames) for j in range(0, 5)]

    def seq_track():
        for ref, trg in track_pairs:
            R.RegisterRGBD360(ctx).RegisterPbMap(ref, trg, 25, R.PLANAR_ODOMETRY_3DoF)

    def bat_track():
        for i in range(5, a.frames):
            batch.track(F[:i], F[i], num_check=5)

    def seq_lc():
        for ref, trg in lc_pairs:
            reg = R.RegisterRGBD360(ctx)
            if reg.RegisterPbMap(ref, trg, 25, R.PLANAR_3DoF) and len(reg.getMatchedPlanes()) > 5 and \
                    reg.getAreaMatched() > 15.0:
                al = R.RegisterPhotoICP(ctx)
                al.params = p
                al.setSourceFrame(ref)
                al.setTargetFrame(trg)
                al.alignFrames360(Ro @ reg.getPose() @ Ri, R.PHOTO_DEPTH)

    def bat_lc():
        for i in range(10, a.frames):
            batch.loop_closures([(F[j], F[i]) for j in range(0, 5)], params=p)

    def bat_lc_all():                           # every frame's candidates in one call
        batch.loop_closures(lc_pairs, params=p)

    def timed(fn):
        fn()                                   # warm-up
        best = 1e30
        for _ in range(a.reps):
            t = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t)
        return best

    out = {"frames": a.frames, "lanes": a.lanes, "sensors": "8x640x480", "data": "synthetic"}
    n_gated = sum(r["dense_rc"] >= 0 for i in range(10, a.frames)
                  for r in batch.loop_closures([(F[j], F[i]) for j in range(0, 5)], params=p))
    for name, s, b, n in (("track", seq_track, bat_track, len(track_pairs)),
                          ("lc", seq_lc, bat_lc, len(lc_pairs))):
        ts, tb = timed(s), timed(b)
        out[name] = {"pairs": n, "sequential_pairs_per_s": n / ts, "batched_pairs_per_s": n / tb,
                     "speedup": ts / tb}
    out["lc"]["refined_pairs"] = int(n_gated)
    out["lc"]["batched_one_call_pairs_per_s"] = len(lc_pairs) / timed(bat_lc_all)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
