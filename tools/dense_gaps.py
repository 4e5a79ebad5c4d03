"""Gaps in the dense queue's ICP launches of a rocprofv3 kernel trace: sorts the k_icp_pass dispatches (the queue's
stream runs nothing else) by start time and reports the idle gaps between one ending and the next starting, the
share of the traced span the dense stream was busy, and the gaps' distribution (batch boundaries are the long ones).
usage: python tools/dense_gaps.py <kernel_trace.csv>"""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_icp_pass" in r["Kernel_Name"]]
st = np.array([int(r["Start_Timestamp"]) for r in rows], np.int64)
en = np.array([int(r["End_Timestamp"]) for r in rows], np.int64)
o = np.argsort(st)
st, en = st[o], en[o]
# merge overlapping intervals (none expected on one stream), then gaps
busy, gaps = 0, []
cur_s, cur_e = st[0], en[0]
for s, e in zip(st[1:], en[1:]):
    if s <= cur_e:
        cur_e = max(cur_e, e)
    else:
        busy += cur_e - cur_s
        gaps.append(s - cur_e)
        cur_s, cur_e = s, e
busy += cur_e - cur_s
span = en.max() - st.min()
g = np.array(gaps, np.float64) * 1e-3   # us
print(f"icp launches {len(st)}  span {span*1e-6:.1f} ms  dense stream busy {busy*1e-6:.1f} ms ({100*busy/span:.1f} %)")
for lo, hi in ((0, 5), (5, 20), (20, 100), (100, 1000), (1000, 1e9)):
    m = (g >= lo) & (g < hi)
    print(f"  gaps {lo:>5}-{hi:<8g} us: {m.sum():6d}  total {g[m].sum()*1e-3:8.1f} ms")
