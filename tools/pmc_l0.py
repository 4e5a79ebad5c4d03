"""Per pair-pass counters of the level-0 ICP pass from a tools/r4_pmc.sh directory: every counter of every level-0
dispatch divided by the dispatch's jobs (SQ_WAVES of the same pass / waves of one job's grid), median over
dispatches; FETCH_SIZE doubled (gfx950 correction, MI355X_MICROARCH.md §HBM).
usage: python tools/pmc_l0.py gpurun_out/pmc4_<tag>"""
import csv
import glob
import json
import os
import re
import sys

import numpy as np

src = sys.argv[1]


def is_l0(name):
    return re.search(r"k_icp_pass<\d+, \d+, 1[,>]", name) is not None or re.search(r"k_icp_passILi\d+ELi\d+ELi1E", name) is not None


per_counter = {}
gx = set()
for f in glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True):
    disp = {}
    for r in csv.DictReader(open(f)):
        if not is_l0(r["Kernel_Name"]):
            continue
        gx.add(int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0))
        disp.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
    waves_per_job = 512 * 4   # 512 workgroups x 4 waves per pair at VGA / HiRes (the capped per-job grid)
    for d in disp.values():
        if not d.get("SQ_WAVES"):
            continue
        jobs = d["SQ_WAVES"] / waves_per_job
        for k, v in d.items():
            if k != "SQ_WAVES":
                per_counter.setdefault(k, []).append(v / jobs)
out = {k: float(np.median(v)) for k, v in per_counter.items()}
if "FETCH_SIZE" in out:
    out["hbm_read_bytes_per_pair_pass"] = 2 * out["FETCH_SIZE"] * 1024
b = json.load(open(os.path.join(src, "dense.json")))
r = b["roofline"]
out.update({"dense_alone_pairs_per_s": b["value"], "avg_launch_ms": r["avg_launch_ms"],
            "pairs_per_launch": r["pairs_per_launch"], "us_per_pair_pass": r["avg_launch_ms"] * 1e3 / r["pairs_per_launch"],
            "frac": r["frac"]})
print(json.dumps(out, indent=1))
