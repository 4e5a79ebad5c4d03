"""Per-kernel duration and GPU area of a rocprofv3 kernel trace: calls, mean duration, mean workgroups per launch and
CU-microseconds per call (duration x min(workgroups, 256): a workgroup per CU as the unit), sorted by area.
usage: python tools/kernel_area.py <kernel_trace.csv> [per=<n calls divisor name>]"""
import collections
import csv
import re
import sys


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?|__amd_\w+)", name)
    return m.group(1) if m else name[:60]


acc = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for r in csv.DictReader(open(sys.argv[1])):
    n = short(r["Kernel_Name"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    wg = (int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])) / max(
        1, int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"]))
    a = acc[n]
    a[0] += 1; a[1] += d; a[2] += wg; a[3] += d * min(wg, 256)
tot = sum(a[3] for a in acc.values())
print(f"{'kernel':34s} {'calls':>6s} {'us/call':>9s} {'WG/call':>8s} {'CU-us/call':>11s} {'area%':>6s}")
for n, a in sorted(acc.items(), key=lambda kv: -kv[1][3]):
    print(f"{n[:34]:34s} {a[0]:6d} {a[1] / a[0]:9.2f} {a[2] / a[0]:8.0f} {a[3] / a[0]:11.0f} {100 * a[3] / tot:6.1f}")
