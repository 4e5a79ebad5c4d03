"""A lone pair on an idle GPU (the reference's sequential callers, OdometryRGBD360.cpp:141-257): wall-clock of
alignFrames360(PHOTO_DEPTH) on two built VGA frames with the bench's schedule (levels 4..1 reference schedule, 20
GN iterations at level 0), its pose (A/B builds must agree bit for bit) and the per-level ICP pass times.
usage: [R360_LIB=...] python tools/lone_align.py [calls]"""
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rgbd360_amd as R  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
ctx = R.Context(0)
cal = R.Calib360(ctx, 480, 640)
cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
seed = 360 << 16
fr = []
for i in range(2):
    b, d = cal.synth_frame(seed, R.synth_path_pose(seed, i))
    f = R.Frame360(cal); f.upload(b, d); f.build(); fr.append(f)
reg = R.RegisterPhotoICP(ctx)
reg.setNumPyr(5); reg.setGrayVariance(3.0 / 255)
reg.params.fixed_iters_level0 = 20
reg.setTargetFrame(fr[0]); reg.setSourceFrame(fr[1])
P = np.eye(4)
for _ in range(3):
    reg.alignFrames360(P, R.PHOTO_DEPTH)
# host cost of enqueueing one alignment (r360_align360_async) and the matching result wait
init = R._mat16(P)
te = []
for _ in range(calls):
    t0 = time.perf_counter()
    R._check(R.lib().r360_align360_async(ctx.h, fr[0].h, fr[1].h, R._fptr(init), R.PHOTO_DEPTH, 0,
                                         R.C.byref(reg.params)), "align async")
    te.append(time.perf_counter() - t0)
    R._check(R.lib().r360_align360_result(ctx.h, None, None, None, None), "align result")
for lv in range(5):
    ctx.kernel_stats(lv)
ctx.kernel_time_reset()
tw = []
for _ in range(calls):   # wall-clock without the per-launch timing events
    t0 = time.perf_counter()
    reg.alignFrames360(P, R.PHOTO_DEPTH)
    tw.append(time.perf_counter() - t0)
ks = [ctx.kernel_stats(lv) for lv in range(5)]
span = sum(k[0] for k in ks) / calls
lvtxt = " ".join(f"L{lv} {k[0] / max(k[1], 1):.2f}us x{k[1] / calls:.0f}" for lv, k in enumerate(ks))
ctx.timing(True); ctx.timing_reset()
t = []
for _ in range(calls):
    t0 = time.perf_counter()
    reg.alignFrames360(P, R.PHOTO_DEPTH)
    t.append(time.perf_counter() - t0)
ms0, n0 = ctx.timing_read("k_icp_pass_L0")
ms1, n1 = ctx.timing_read("k_icp_pass")
ctx.timing(False)
pose = np.asarray(reg.getOptimalPose(), dtype=np.float32)
print(f"lib {os.path.basename(R.LIB_PATH)}: align {1e3 * np.median(tw):.3f} ms median ({1e3 * min(tw):.3f} min) per lone pair"
      f" ({1e3 * np.median(t):.3f} ms with timing events);"
      f" level-0 pass {1e3 * ms0 / max(n0, 1):.2f} us x {n0 / calls:.1f}, coarse pass {1e3 * ms1 / max(n1, 1):.2f} us x"
      f" {n1 / calls:.1f} per pair (event-timed); pose sha {hashlib.sha1(pose.tobytes()).hexdigest()[:12]}")
print(f"  in-kernel spans per pair {1e-3 * span:.3f} ms ({lvtxt}); host enqueue {1e6 * np.median(te):.1f} us")
