"""Host cost of kernel launches from a rocprofv3 --hip-trace --kernel-trace run: per kernel name (joined by
correlation id), the count and mean / median duration of the hipLaunchKernel call that enqueued it.
usage: python tools/launch_cost.py <hip_api_trace.csv> <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

import numpy as np

api = {}
for r in csv.DictReader(open(sys.argv[1])):
    if "Launch" in r["Function"]:
        api[r["Correlation_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
per = defaultdict(list)
for r in csv.DictReader(open(sys.argv[2])):
    c = r["Correlation_Id"]
    if c in api:
        per[r["Kernel_Name"].split("(")[0][:60]].append(api[c])
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))[:15]:
    v = np.array(v)
    print(f"{k:62s} n {len(v):6d}  mean {v.mean():7.2f} us  median {np.median(v):7.2f} us  total {v.sum()*1e-3:8.1f} ms")
