"""Per-stage timing of the plane half + PbMap registration on a synthetic VGA pair (debug aid)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rgbd360_amd as R

ctx = R.Context(0)
cal = R.Calib360(ctx, 480, 640)
cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
seed = 360 << 16
A = R.synth_path_pose(seed, 0)
B = R.synth_path_pose(seed, 1)
fr = []
for P in (A, B):
    b, d = cal.synth_frame(seed, P)
    f = R.Frame360(cal)
    f.upload(b, d)
    fr.append(f)
lib = R.lib()
lib.r360_ctx_timing(ctx.h, 1)
for it in range(6):
    t0 = time.perf_counter()
    for f in fr:
        f.build(R.BUILD_UNDISTORT | R.BUILD_PLANES)
    t1 = time.perf_counter()
    reg = R.RegisterRGBD360(ctx)
    ok = reg.RegisterPbMap(fr[0], fr[1], 25, R.PLANAR_3DoF)
    t2 = time.perf_counter()
    print(f"iter {it}: 2 frame plane builds {1e3*(t1-t0):.2f} ms, RegisterPbMap {1e3*(t2-t1):.2f} ms ok={ok} "
          f"planes {len(fr[0].planes())}/{len(fr[1].planes())} matches {len(reg.getMatchedPlanes())}")
    if it == 1:
        lib.r360_ctx_timing_reset(ctx.h)
names = ["k_cloud", "k_bilateral", "k_dcm", "k_distmap", "k_normals", "k_ccl", "k_plane_fit", "k_refine", "k_model_stats"]
for n in names:
    ms, cnt = C_ms = R.C.c_double(), R.C.c_long()
    lib.r360_ctx_timing_read(ctx.h, n.encode(), R.C.byref(ms), R.C.byref(cnt))
    if cnt.value:
        print(f"  {n:14s} {1e3*ms.value/cnt.value:9.1f} us/launch-group  (n={cnt.value})")
