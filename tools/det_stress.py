"""GPU diagnostic: run-to-run determinism of queued (batched) dense alignments.  Reference: the unqueued records of
pairs [0, N); then `reps` queued runs (16 pipelines, dense queue) of the same pairs; prints the mismatching pairs per
run.  R360_LIB selects the library (missing newer entry points are skipped, so older builds load too)."""
import sys, os, ctypes
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import rgbd360_amd as R
_L = ctypes.CDLL(R.LIB_PATH)
R._SIGS[:] = [s for s in R._SIGS if hasattr(_L, s[0])]
from rgbd360_amd import odometry as OD
N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 3
SEED = 360 << 16
rt8 = np.stack([np.loadtxt(f"{R.EXTRINSICS_DIR}/Rt_0{k + 1}.txt", dtype=np.float32) for k in range(8)])
bgr = np.zeros((N + 1, 8, 480, 640, 3), np.uint8); dep = np.zeros((N + 1, 8, 480, 640), np.uint16)
for i in range(N + 1):
    bgr[i], dep[i] = R.synth_frame_rt(480, 640, rt8, SEED, R.synth_path_pose(SEED, i))
pin = R.HostPinned(bgr, dep)
p = R.IcpParams.default(); p.n_pyr = 5; p.std_dev_photo = np.float32(3.0 / 255); p.fixed_iters_level0 = 20
r0 = OD.SequenceRunner(0, 480, 640, 16, p)
ref = np.zeros((1, N, OD.REC), np.float32); r0.run(0, N, lambda i: (bgr[i], dep[i]), ref); r0.close()
print("lib", os.path.basename(R.LIB_PATH), "pairs", N, "depth", depth, flush=True)
for k in range(reps):
    rn = OD.SequenceRunner(0, 480, 640, 16, p, queue=16, depth=depth)
    rec = np.zeros((1, N, OD.REC), np.float32); rn.run(0, N, lambda i: (bgr[i], dep[i]), rec)
    st = rn.queue.stats(); rn.close()
    bad = [i for i in range(N) if not np.array_equal(rec[0, i], ref[0, i])]
    print(f"run {k}: {len(bad)} mismatching pairs {bad[:10]} (batches {st['batches']})", flush=True)
pin.close()
