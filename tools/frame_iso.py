"""Frame builds one at a time on an idle GPU (every stage: undistort, plane stage, stitch, pyramid, compaction), for
isolated per-kernel durations under rocprofv3 --kernel-trace --stats.
usage: python tools/frame_iso.py [frames] [rows cols]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rgbd360_amd as R  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
rows, cols = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (480, 640)
ctx = R.Context(0)
cal = R.Calib360(ctx, rows, cols)
cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
seed = 360 << 16
b, d = cal.synth_frame(seed, R.synth_path_pose(seed, 0))
f = R.Frame360(cal)
flags = R.BUILD_UNDISTORT | R.BUILD_PLANES | R.BUILD_SPHERE | R.BUILD_PYRAMID
t = []
for i in range(n):
    f.upload(b, d)
    t0 = time.perf_counter()
    f.build(flags)
    t.append(time.perf_counter() - t0)
t.sort()
print(f"frame build {rows}x{cols}: median {1e3 * t[len(t) // 2]:.3f} ms, min {1e3 * t[0]:.3f} ms over {n}")
