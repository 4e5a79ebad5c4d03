"""GPU occupancy of a rocprofv3 kernel trace: wall span, time with >= 1 kernel running, mean kernel
concurrency, and per-kernel totals, over the last <window_ms> of the trace (the bench's timed region).
usage: python tools/busy.py <kernel_trace.csv> <window_ms> [top kernels, default 25]"""
import csv
import collections
import re
import sys


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?|__amd_\w+)", name)
    return m.group(1) if m else name[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows]
ev.sort()
t0, t1 = ev[0][0], max(e[1] for e in ev)
ts = t1 - float(sys.argv[2]) * 1e6
ev = [e for e in ev if e[0] >= ts]
t0 = ev[0][0]
pts = sorted([(s, 1) for s, _, _ in ev] + [(e, -1) for _, e, _ in ev])
busy = conc = 0.0
cur, last = 0, t0
for t, d in pts:
    if cur > 0:
        busy += t - last
        conc += cur * (t - last)
    cur += d
    last = t
span = t1 - t0
print(f"span {span / 1e6:.2f} ms  busy(>=1 kernel) {busy / 1e6:.2f} ms ({100 * busy / span:.1f}%)  "
      f"mean concurrency while busy {conc / max(busy, 1):.2f}")
tot = collections.Counter()
cnt = collections.Counter()
for s, e, n in ev:
    tot[n] += e - s
    cnt[n] += 1
TOP = int(sys.argv[3]) if len(sys.argv) > 3 else 25
for n, v in tot.most_common(TOP):
    print(f"{v / 1e6:9.2f} ms  {cnt[n]:6d} x {v / cnt[n] / 1e3:8.2f} us  {n}")

# per-kernel grid sizes (workgroups) of the window, to tell full-GPU kernels from latency-bound ones
wg = collections.defaultdict(set)
for r in rows:
    if int(r["Start_Timestamp"]) >= ts:
        try:
            g = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
            w = int(r["Workgroup_Size_X"]) * int(r.get("Workgroup_Size_Y", 1) or 1) * int(r.get("Workgroup_Size_Z", 1) or 1)
            wg[short(r["Kernel_Name"])].add(g // max(w, 1))
        except (KeyError, ValueError):
            pass
print("workgroups per launch:")
for n, v in tot.most_common(TOP):
    print(f"  {n:28s} {sorted(wg[n])[:6]}")
