"""Per-kernel share of GPU occupancy from one rocprofv3 --pmc pass (SQ_WAVE_CYCLES = summed wave lifetimes,
SQ_BUSY_CU_CYCLES, SQ_INSTS_VALU, SQ_WAVES): which kernels hold the CUs, not just which run longest.
usage: python tools/pmc_kernels.py <dir with *counter_collection.csv> [top]"""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?|__amd_\w+)", name)
    return m.group(1) if m else name[:60]


agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
tot = {c: sum(v.get(c, 0.0) for v in agg.values()) for c in ("SQ_WAVE_CYCLES", "SQ_BUSY_CU_CYCLES", "SQ_INSTS_VALU")}
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
print(f"{'kernel':32s} {'disp':>6s} {'waves/d':>9s} {'wave-cyc %':>10s} {'busyCU %':>9s} {'VALU %':>7s} {'wcyc/d':>11s}")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:top]:
    n = max(len(disp[k]), 1)
    pc = lambda c: 100 * v.get(c, 0) / tot[c] if tot.get(c) else 0.0
    print(f"{k:32s} {n:6d} {v.get('SQ_WAVES', 0) / n:9.0f} {pc('SQ_WAVE_CYCLES'):10.2f} {pc('SQ_BUSY_CU_CYCLES'):9.2f} "
          f"{pc('SQ_INSTS_VALU'):7.2f} {v.get('SQ_WAVE_CYCLES', 0) / n:11.0f}")
