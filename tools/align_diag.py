"""Diagnostic: alignFrames360 on the synthetic VGA pair of tests/test_gpu_dense.py (reference schedule),
GPU vs oracle iterations per level and final pose difference; also the oracle's own sensitivity to a
1e-7 rad perturbation of the initial pose."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rgbd360_amd as R  # noqa: E402
from oracle import oracle360 as O  # noqa: E402

ctx = R.Context(0)
cal = R.Calib360(ctx, 480, 640)
cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
seed = 360 << 16
A = R.synth_path_pose(seed, 0)
rel = np.eye(4, dtype=np.float32)
a = np.deg2rad(4.0)
rel[1:3, 1:3] = [[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]]
rel[:3, 3] = [0, 0.25, 0.15]
b1, d1 = cal.synth_frame(seed, A)
b2, d2 = cal.synth_frame(seed, A @ rel)
f1, f2 = R.Frame360(cal), R.Frame360(cal)
f1.upload(b1, d1); f2.upload(b2, d2)
f1.build(); f2.build()
reg = R.RegisterPhotoICP(ctx)
reg.setNumPyr(5); reg.setGrayVariance(3.0 / 255)
reg.setTargetFrame(f1); reg.setSourceFrame(f2)
s1b, s1d = f1.sphere(); s2b, s2d = f2.sphere()
p = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255))
for init_tw in (0.0, 1e-7, -1e-7):
    init = O.exp_se3([0, 0, 0, init_tw, 0, 0], pseudo=False).astype(np.float32)
    reg.alignFrames360(init, R.PHOTO_DEPTH)
    rco, pose, H, g, st = O.align360(s1b, s1d, s2b, s2d, init, O.PHOTO_DEPTH, p)
    gp = reg.getOptimalPose()
    dr = O.rot_angle(gp[:3, :3], pose[:3, :3]); dt = float(np.linalg.norm(gp[:3, 3] - pose[:3, 3]))
    print(f"init tweak {init_tw:+.0e}: gpu iters {list(reg.stats.iters[:5])} evals {list(reg.stats.evals[:5])} | "
          f"oracle iters {list(st.iters[:5])} evals {list(st.evals[:5])} | dR {dr:.2e} dt {dt:.2e}")
    if init_tw == 0.0:
        P0 = pose
    else:
        print(f"   oracle vs oracle(tweak 0): dR {O.rot_angle(pose[:3, :3], P0[:3, :3]):.2e} "
              f"dt {float(np.linalg.norm(pose[:3, 3] - P0[:3, 3])):.2e}")

# error-value agreement of the fused pass at a few poses (relative difference of err2 GPU vs oracle)
lt, ls = f1.level(0), f2.level(0)
for P in (np.eye(4, dtype=np.float32), rel.astype(np.float32), np.linalg.inv(rel).astype(np.float32)):
    H, gg, e2, nv, nvis = reg.eval(0, P, R.PHOTO_DEPTH)
    e, e2r, nvr = O.error_sphere(ls, lt, P, O.PHOTO_DEPTH, p)
    Hr, gr, nvisr = O.hessgrad_sphere(ls, lt, P, O.PHOTO_DEPTH, p)
    print(f"eval: err2 rel diff {(e2 - e2r) / e2r:+.3e}  counts {nv - nvr} {nvis - nvisr}  "
          f"H max rel {np.abs(H - Hr).max() / np.abs(Hr).max():.2e}")
