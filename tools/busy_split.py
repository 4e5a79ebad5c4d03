"""Per (kernel, workgroups per launch) totals of a rocprofv3 kernel trace over the last <window_ms>: which launch
sizes of a multi-size kernel (the pyramid levels, the ICP levels) take the time.
usage: python tools/busy_split.py <kernel_trace.csv> <window_ms> <name substring> [...]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
t1 = max(int(r["End_Timestamp"]) for r in rows)
ts = t1 - float(sys.argv[2]) * 1e6
keys = sys.argv[3:]
tot, cnt = collections.Counter(), collections.Counter()
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < ts:
        continue
    name = r["Kernel_Name"]
    if not any(k in name for k in keys):
        continue
    m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
    n = m.group(1) if m else name[:40]
    g = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
    w = int(r["Workgroup_Size_X"]) * int(r.get("Workgroup_Size_Y", 1) or 1) * int(r.get("Workgroup_Size_Z", 1) or 1)
    k = (n, g // max(w, 1))
    tot[k] += e - s
    cnt[k] += 1
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{v / 1e6:9.2f} ms  {cnt[k]:6d} x {v / cnt[k] / 1e3:8.2f} us  {k[0]}  wg {k[1]}")
