"""GPU diagnostic: the test_gpu_sequence scenario as a loop (256-frame sequence, unqueued 16-pipeline reference over
255 pairs; queued 16-pipeline runs over all pairs at depth 1 / 3 and the 7/8 shard on 5 pipelines), printing
mismatching pairs and which record fields differ."""
import sys, os, ctypes
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import rgbd360_amd as R
_L = ctypes.CDLL(R.LIB_PATH)
R._SIGS[:] = [s for s in R._SIGS if hasattr(_L, s[0])]
from rgbd360_amd import odometry as OD
SEED = 360 << 16
rt8 = np.stack([np.loadtxt(f"{R.EXTRINSICS_DIR}/Rt_0{k + 1}.txt", dtype=np.float32) for k in range(8)])
bgr = np.zeros((256, 8, 480, 640, 3), np.uint8); dep = np.zeros((256, 8, 480, 640), np.uint16)
for i in range(256):
    bgr[i], dep[i] = R.synth_frame_rt(480, 640, rt8, SEED, R.synth_path_pose(SEED, i))
pin = R.HostPinned(bgr, dep)
p = R.IcpParams.default(); p.n_pyr = 5; p.std_dev_photo = np.float32(3.0 / 255); p.fixed_iters_level0 = 20
fix = OD.SequenceRunner(0, 480, 640, 16, p)
ref = np.zeros((1, 255, OD.REC), np.float32); fix.run(0, 255, lambda i: (bgr[i], dep[i]), ref); ref = ref[0]
def summ(rec, r0, r1):
    out = []
    for i in range(r1 - r0):
        d = np.nonzero(rec[i] != ref[r0 + i])[0]
        if len(d):
            out.append((r0 + i, int((d < 16).sum()), int(((d >= 16) & (d < 52)).sum()), [int(k) for k in d[d >= 52]]))
    return out
print("lib", os.path.basename(R.LIB_PATH), flush=True)
ref2 = np.zeros((1, 255, OD.REC), np.float32); fix.run(0, 255, lambda i: (bgr[i], dep[i]), ref2)
print("unqueued again:", summ(ref2[0], 0, 255)[:6], flush=True)
for k in range(3):
    for depth in (1, 3):
        rn = OD.SequenceRunner(0, 480, 640, 16, p, queue=16, depth=depth)
        rec = np.zeros((1, 255, OD.REC), np.float32); rn.run(0, 255, lambda i: (bgr[i], dep[i]), rec); rn.close()
        b = summ(rec[0], 0, 255)
        print(f"round {k} queued 16 depth {depth}: {len(b)} bad {b[:6]}", flush=True)
    p0, p1 = OD.shard_pairs(7, 8)
    rn = OD.SequenceRunner(0, 480, 640, 5, p, queue=16, depth=3)
    rec = np.zeros((3, p1 - p0, OD.REC), np.float32)
    rn.run(p0, p1, lambda i: (bgr[i], dep[i]), rec, repeats=3, runs=OD.split_range(p0, p1, 5)); rn.close()
    for r in range(3):
        b = summ(rec[r], p0, p1)
        print(f"round {k} shard 7/8 repeat {r}: {len(b)} bad {b[:6]}", flush=True)
fix.close(); pin.close()
