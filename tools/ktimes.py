"""Summarise a rocprofv3 kernel trace by (kernel, grid size): python tools/ktimes.py <trace.csv>"""
import collections
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
g = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[-28:]
    g[(name, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
tot = sum(sum(v) for v in g.values())
for k in sorted(g, key=lambda k: -sum(g[k])):
    v = np.array(g[k])
    print(f"{k[0]:28s} grid {k[1]:8d} n {len(v):4d} median {np.median(v):7.1f} us  min {v.min():7.1f}  max {v.max():7.1f}  total {v.sum()/1e3:7.2f} ms ({100*v.sum()/tot:4.1f}%)")
