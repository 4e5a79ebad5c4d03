"""Per-alignment timeline of a tools/lone_trace2.sh trace: the alignments are the runs of ICP pass launches between
the state uploads (H2D copies); prints, per alignment, the H2D copy, the first kernel's start, the kernels' busy
time, the gaps between kernels and the D2H copy, in us.
usage: python tools/lone_timeline.py <trace dir>"""
import csv
import glob
import sys

import numpy as np

d = sys.argv[1]
kf = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
mf = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
ev = []
for r in csv.DictReader(open(kf)):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:40]))
if mf:
    for r in csv.DictReader(open(mf[0])):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "C"), ""))
ev.sort()
# alignments: a host-to-device copy followed by k_icp_pass launches, up to the next device-to-host copy
rows = []
i = 0
while i < len(ev):
    s, e, kind, name = ev[i]
    if "HOST_TO_DEVICE" in kind or kind == "H2D":
        j = i + 1
        ks = []
        while j < len(ev) and ev[j][2] == "K":
            ks.append(ev[j]); j += 1
        if j < len(ev) and ("DEVICE_TO_HOST" in ev[j][2] or ev[j][2] == "D2H") and len(ks) > 30:
            d2h = ev[j]
            busy = sum(k[1] - k[0] for k in ks)
            gaps = [ks[t + 1][0] - ks[t][1] for t in range(len(ks) - 1)]
            rows.append((e - s, ks[0][0] - e, busy, sum(gaps), np.median(gaps), d2h[0] - ks[-1][1], d2h[1] - d2h[0],
                         d2h[1] - s, len(ks)))
        i = j
    else:
        i += 1
if not rows:
    print("no alignments found;", len(ev), "events; kinds", sorted(set(x[2] for x in ev))[:10])
    sys.exit(0)
a = np.array(rows, dtype=float) / 1e3
a[:, 8] *= 1e3
print("per alignment (us): h2d copy | h2d end -> 1st kernel | kernels busy | sum gaps | median gap | last kernel -> d2h start | d2h | h2d start -> d2h end | kernels")
for r in a[-10:]:
    print(" ".join(f"{x:8.1f}" for x in r))
print("median:", " ".join(f"{x:8.1f}" for x in np.median(a, axis=0)))
