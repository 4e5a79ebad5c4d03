"""A/B of the level-0 pass form for lone alignments (experiment library, R360_ICP_PF): the poses of default-parameter
alignFrames360 calls over consecutive synthetic frames, printed with a hash so two runs can be compared.
usage: R360_LIB=rgbd360_amd/lib/librgbd360_hip_exp.so R360_ICP_PF=5|6 python tools/pf_ab.py"""
import hashlib
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
for i in range(1, 6):
    b, d = cal.synth_frame(seed, R.synth_path_pose(seed, i))
    f = R.Frame360(cal); f.upload(b, d); f.build(); fr.append(f)
reg = R.RegisterPhotoICP(ctx)
reg.setNumPyr(5); reg.setGrayVariance(3.0 / 255)
for k in range(1, len(fr)):
    reg.setTargetFrame(fr[k - 1]); reg.setSourceFrame(fr[k])
    for fixed in (0, 20):
        reg.params.fixed_iters_level0 = fixed
        reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH)
        P = np.asarray(reg.getOptimalPose(), dtype=np.float32)
        print(f"pair {k} fixed {fixed}: sha {hashlib.sha1(P.tobytes()).hexdigest()[:12]} t {P[:3, 3]}")
    for lv in range(5):
        H, g, e2, nv, nvis = reg.eval(lv, np.eye(4, dtype=np.float32), R.PHOTO_DEPTH)
        s = np.concatenate([H.ravel(), g, [e2, nv, nvis]])
        print(f"  eval L{lv} sha {hashlib.sha1(s.tobytes()).hexdigest()[:12]} e2 {e2!r} H00 {H[0, 0]!r}")
