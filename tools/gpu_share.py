"""Capacity-weighted GPU time per kernel from a rocprofv3 kernel trace: each dispatch is weighted by the
fraction of the chip's wave slots its grid can occupy (waves in the grid / resident-wave capacity at the
kernel's VGPR count), so long-running narrow kernels (8 workgroups) and full-chip passes compare on
the same scale.  usage: python tools/gpu_share.py <kernel_trace.csv> [window_ms] [n_pairs]"""
import csv
import collections
import re
import sys

CUS, SIMDS, VGPRS = 256, 4, 512


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?|__amd_\w+)", name)
    return m.group(1) if m else name[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) if len(sys.argv) > 2 else 0
npairs = float(sys.argv[3]) if len(sys.argv) > 3 else 0
t_end = max(int(r["End_Timestamp"]) for r in rows)
agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
t_min = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if win and s < t_end - win * 1e6:
        continue
    t_min = s if t_min is None else min(t_min, s)
    grid = 1
    for ax in "XYZ":
        grid *= int(r.get("Grid_Size_" + ax, 1) or 1)
    vg = int(r.get("Arch_VGPR_Count", r.get("VGPR_Count", 0)) or 0) or 32
    waves = max(1, (grid + 63) // 64)
    per_simd = max(1, min(8, VGPRS // max(vg, 8)))
    cap = CUS * SIMDS * per_simd
    frac = min(1.0, waves / cap)
    d = (e - s) / 1e3
    a = agg[short(r["Kernel_Name"])]
    a[0] += d; a[1] += d * frac; a[2] += 1
span = (t_end - t_min) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"span {span / 1e3:.2f} ms   capacity-weighted kernel time {tot / 1e3:.2f} ms ({100 * tot / span:.1f}% of the chip)")
for k, (d, w, n) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    per = f"  {w / npairs:8.1f} us/pair" if npairs else ""
    print(f"{k:32s} {n:6d} x {d / n:8.1f} us  weighted {w / 1e3:8.2f} ms ({100 * w / span:5.1f}%){per}")
