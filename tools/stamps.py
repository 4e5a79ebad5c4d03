"""Diagnostic: in-kernel stamps of the last ICP pass per level (needs the -DR360_STAMPS library:
`make -C rgbd360_amd/csrc stamps`, run with R360_LIB=rgbd360_amd/lib/librgbd360_hip_stamps.so)."""
import ctypes as C
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
reg.setTargetFrame(fr[0]); reg.setSourceFrame(fr[1])
P = np.eye(4, dtype=np.float32)
for lv in (4, 3, 2, 1, 0):
    for rep in range(4):
        reg.eval(lv, P, R.PHOTO_DEPTH)
    st = (C.c_ulonglong * 12)()
    R.lib().r360_ctx_debug_stamps(ctx.h, st)
    t = np.array(list(st), dtype=np.uint64).astype(np.float64)
    # grid-wide first start / last loop end from the per-workgroup stamps of this level's last pass
    nbl = min(512, -(-fr[0].level(lv)["gray"].size // 256))
    bs = (C.c_ulonglong * (3 * 8192))()
    R.lib().r360_debug_block_stamps(bs, 8192)
    ab = np.array(list(bs), dtype=np.float64).reshape(3, 8192)[:2, :nbl]
    base = ab[0].min()
    us = lambda x: (x - base) / 100.0
    print(f"level {lv} ({nbl} wg): all-blocks loop end {us(ab[1].max()):7.2f} | last block: start {us(t[0]):7.2f} loop-end {us(t[1]):7.2f}"
          f" ticket {us(t[2]):7.2f} records {us(t[3]):7.2f} end {us(t[4]):7.2f}  (us from first block start)")

# per-workgroup start / loop-end distribution of the last level-0 pass
nb = int(os.environ.get("NB", "768"))
buf = (C.c_ulonglong * (3 * 8192))()
R.lib().r360_debug_block_stamps(buf, 8192)
a = np.array(list(buf), dtype=np.float64).reshape(3, 8192)[:2, :nb]
hwid = np.array(list(buf), dtype=np.uint64).reshape(3, 8192)[2, :nb]
t0 = a[0].min()
st, en = (a[0] - t0) / 100.0, (a[1] - t0) / 100.0
q = lambda x: " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 10, 50, 90, 100]))
print("block start   pct 0/10/50/90/100:", q(st))
print("block loopend pct 0/10/50/90/100:", q(en))
print("block busy    pct 0/10/50/90/100:", q(en - st))
m = a[0] > 0
b = np.nonzero(m)[0]
busy = (a[1] - a[0])[m] / 100.0
print("blocks used", len(b))
for x in range(8):
    sel = (b % 8) == x
    print(f"xcd {x}: busy pct 0/50/100 {np.percentile(busy[sel], [0, 50, 100]).round(2)}")
# workgroups per CU (HW_ID: CU_ID bits 8-11, SH_ID 12, SE_ID 13-15; XCC_ID in the high word) and busy time
hw = hwid[m]
cu_key = ((hw >> np.uint64(32)) << np.uint64(8)) | ((hw >> np.uint64(8)) & np.uint64(0xff))
keys, inv, counts = np.unique(cu_key, return_inverse=True, return_counts=True)
per_blk = counts[inv]
print(f"CUs used {len(keys)}; workgroups per CU: " + ", ".join(f"{k}: {int((counts == k).sum())} CUs" for k in np.unique(counts)))
for k in np.unique(per_blk):
    print(f"  blocks on CUs holding {k}: busy mean {busy[per_blk == k].mean():6.2f} max {busy[per_blk == k].max():6.2f}")
order = np.argsort(a[0][m])
k = len(order)
for part in range(4):
    sl = order[part * k // 4:(part + 1) * k // 4]
    print(f"start-quartile {part}: busy mean {busy[sl].mean():6.2f}")

# align mode (device Gauss-Newton step in the last workgroup): stamps of the final level-0 pass, beside an eval pass
# at the aligned pose (same pixels, no GN step)
def last_pass(label, nbl=512):
    st = (C.c_ulonglong * 12)()
    R.lib().r360_ctx_debug_stamps(ctx.h, st)
    t = np.array(list(st), dtype=np.uint64).astype(np.float64)
    bs = (C.c_ulonglong * (3 * 8192))()
    R.lib().r360_debug_block_stamps(bs, 8192)
    ab = np.array(list(bs), dtype=np.float64).reshape(3, 8192)[:2, :nbl]
    base = ab[0].min()
    us = lambda x: (x - base) / 100.0
    le = (ab[1] - base) / 100.0
    print(f"{label}: loop end pct 0/50/90/100 {np.percentile(le, [0, 50, 90, 100]).round(2)} | last block: start"
          f" {us(t[0]):6.2f} loop-end {us(t[1]):6.2f} ticket {us(t[2]):6.2f} records {us(t[3]):6.2f} end {us(t[4]):6.2f}"
          f" | GN state {us(t[7]):6.2f} rank {us(t[10]):6.2f} solve {us(t[11]):6.2f}")


if os.environ.get("ALIGN"):
    reg.params.fixed_iters_level0 = 20
    for rep in range(3):
        reg.alignFrames360(P, R.PHOTO_DEPTH)
    last_pass("align last L0 pass")
    Pa = np.asarray(reg.getOptimalPose(), dtype=np.float32)
    for rep in range(4):
        reg.eval(0, Pa, R.PHOTO_DEPTH)
    last_pass("eval at aligned pose")
