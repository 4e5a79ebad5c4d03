"""Per hardware queue of a rocprofv3 kernel trace (last <window_ms>): kernels, busy ms, and the plane chain per frame
(k_plane_begin start -> k_plane_publish end on the same queue), to compare pipeline schedules.
usage: python tools/queue_busy.py <kernel_trace.csv> <window_ms>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
qk = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get(qk, "0"),
             r.get("Stream_Id", "?")) for r in rows)
t1 = max(e[1] for e in ev)
ts = t1 - float(sys.argv[2]) * 1e6
ev = [e for e in ev if e[0] >= ts]
per = collections.defaultdict(list)
for e in ev:
    per[(e[3], e[4])].append(e)
chains = []
print(f"queue key {qk}; queues {len(per)}")
for k, L in sorted(per.items(), key=lambda kv: -len(kv[1])):
    busy = sum(e[1] - e[0] for e in L) / 1e6
    names = collections.Counter("icp" if "k_icp" in e[2] else "plane" if "plane" in e[2] or "ccl" in e[2] else "other"
                                for e in L)
    beg = None
    for e in L:
        if "k_plane_begin" in e[2]:
            beg = e[0]
        elif "k_plane_publish" in e[2] and beg is not None:
            chains.append((e[1] - beg) / 1e6)
            beg = None
    print(f"  q {k}: {len(L)} kernels {dict(names)} busy {busy:.1f} ms")
if chains:
    chains.sort()
    print(f"plane chain per frame (begin->publish): n {len(chains)} median {chains[len(chains)//2]:.3f} ms "
          f"p90 {chains[int(len(chains)*0.9)]:.3f} mean {sum(chains)/len(chains):.3f}")
