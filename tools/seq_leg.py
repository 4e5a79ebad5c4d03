"""The sequential caller's leg alone (bench.sequential_leg: one pipeline, one pair at a time), for a kernel trace
of a lone frame's chain.  usage: python tools/seq_leg.py [pairs] [plane_batch: -1 = runner default]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import rgbd360_amd as R  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 32
pb = int(sys.argv[2]) if len(sys.argv) > 2 else -1
rt8 = np.stack([np.loadtxt(f"{R.EXTRINSICS_DIR}/Rt_0{k + 1}.txt", dtype=np.float32) for k in range(8)])
n = pairs + 8
BGR = np.zeros((n, 8, 480, 640, 3), np.uint8)
DEP = np.zeros((n, 8, 480, 640), np.uint16)
for j in range(n):
    BGR[j], DEP[j] = R.synth_frame_rt(480, 640, rt8, bench.SEED, R.synth_path_pose(bench.SEED, j))
pin = R.HostPinned(BGR, DEP)   # page-locked, as the bench's inputs (pageable copies are synchronous host staging)
p = R.IcpParams.default()
p.n_pyr = 5
p.std_dev_photo = np.float32(3.0 / 255)
p.fixed_iters_level0 = 20
out = bench.sequential_leg(0, 480, 640, 0, lambda i: (BGR[i], DEP[i]), p, pairs=pairs,
                           plane_batch=None if pb < 0 else pb)
print(json.dumps(out))
