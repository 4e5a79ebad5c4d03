"""Level-0 in-kernel span per pass: eval passes (no GN step) at identity and at the aligned pose vs the passes of
alignFrames360 itself, on one ctx and the same two VGA frames.  usage: python tools/eval_vs_align.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rgbd360_amd as R  # noqa: E402

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
for _ in range(3):
    reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH)
Pa = np.asarray(reg.getOptimalPose(), dtype=np.float32)


def span(fn, n):
    ctx.kernel_time_reset()
    for _ in range(n):
        fn()
    us, launches, ran = ctx.kernel_stats(0)
    return us / max(ran, 1), launches, ran


for name, fn, n in (("eval identity", lambda: reg.eval(0, np.eye(4, dtype=np.float32), R.PHOTO_DEPTH), 40),
                    ("eval aligned", lambda: reg.eval(0, Pa, R.PHOTO_DEPTH), 40),
                    ("align (20 iters)", lambda: reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH), 4),
                    ("eval identity", lambda: reg.eval(0, np.eye(4, dtype=np.float32), R.PHOTO_DEPTH), 40)):
    us, nl, nr = span(fn, n)
    print(f"{name:18s}: level-0 in-kernel span {us:6.2f} us per pass ({nl} launches, {nr} passes ran)")
