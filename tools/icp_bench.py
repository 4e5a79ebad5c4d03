"""Micro-benchmark of the fused ICP pass at each pyramid level (eval mode, HIP-event timed).
usage: R360_LIB=rgbd360_amd/lib/librgbd360_hip_exp.so python tools/icp_bench.py [reps]   (env R360_ICP_PF /
R360_ICP_CAP select variants; experiment build only: make -C rgbd360_amd/csrc exp)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rgbd360_amd as R  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
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
reg.setTargetFrame(fr[0]); reg.setSourceFrame(fr[1])
P = np.eye(4, dtype=np.float32)
if os.environ.get("POSE") == "path":   # the synthetic path's true relative motion between the two frames
    P0, P1 = (np.asarray(R.synth_path_pose(seed, i), dtype=np.float64).reshape(4, 4) for i in range(2))
    P = (np.linalg.inv(P0) @ P1).astype(np.float32)
tag = f"PF={os.environ.get('R360_ICP_PF', 'dflt')} CAP={os.environ.get('R360_ICP_CAP', 'dflt')}"
for lv in [int(x) for x in os.environ.get("LEVELS", "0,1,2").split(",")]:
    for _ in range(3):
        reg.eval(lv, P, R.PHOTO_DEPTH)
    ctx.timing(True); ctx.timing_reset()
    for _ in range(reps):
        H, g, e2, nv, nvis = reg.eval(lv, P, R.PHOTO_DEPTH)
    ms, n = ctx.timing_read("k_icp_pass_L0" if lv == 0 else "k_icp_pass")
    ctx.timing(False)
    N = fr[0].level(lv)["gray"].size
    B = 8 * N + 24 * nvis
    print(f"{tag} level {lv}: {1e3 * ms / n:8.2f} us/pass  {B / (ms / n * 1e-3) / 1e9:8.1f} GB/s algorithmic  (N={N}, V={nvis})")
