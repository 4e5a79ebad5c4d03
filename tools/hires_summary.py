"""HiRes (config 5) PMC summary of tools/prof_r3.sh: level-0 ICP pass counters per pair-pass (each
dispatch's counter / the pairs it ran, Grid_Size_Y of its kernel-trace row), HBM bytes per pair-pass with the gfx950
FETCH_SIZE correction, against the algorithmic 8 N + 24 V of the bench line run beside it.
usage: python tools/hires_summary.py <prof_dir>/hires <hires bench line file>"""
import csv
import glob
import json
import os
import re
import sys

import numpy as np

src, bench_file = sys.argv[1], sys.argv[2]


def is_l0(name):
    return re.search(r"k_icp_pass<\d+, \d+, 1[,>]", name) is not None or re.search(r"k_icp_passILi\d+ELi\d+ELi1E", name) is not None


per = {}
grid = 0
for d in glob.glob(os.path.join(src, "pmc*")):
    jobs = {}   # dispatch -> pairs in the launch (blockIdx.y = job), from the pass's own kernel trace
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            if is_l0(r["Kernel_Name"]):
                jobs[r["Dispatch_Id"]] = int(r["Grid_Size_Y"])
                grid = max(grid, int(r["Grid_Size_X"]))
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if is_l0(r["Kernel_Name"]) and r["Dispatch_Id"] in jobs:
                per.setdefault((d, r["Dispatch_Id"]), {"jobs": jobs[r["Dispatch_Id"]]})[r["Counter_Name"]] = \
                    float(r["Counter_Value"])
waves_per_job = grid // 64 if grid else None


def med(name):
    v = [d[name] / d["jobs"] for d in per.values() if name in d and d["jobs"] > 0]
    return float(np.median(v)) if v else None


out = {"kernel": "k_icp_pass<PHOTO_DEPTH> level 0, config 5 (8 x 1280x960)", "grid_threads": grid,
       "waves_per_job": waves_per_job, "dispatches": len(per)}
for k in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
          "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE"):
    out[k + "_per_pair_pass"] = med(k)
if out["FETCH_SIZE_per_pair_pass"] is not None and out["WRITE_SIZE_per_pair_pass"] is not None:
    out["hbm_bytes_per_pair_pass"] = 2 * out["FETCH_SIZE_per_pair_pass"] * 1024 + out["WRITE_SIZE_per_pair_pass"] * 1024
try:
    line = [l for l in open(bench_file) if l.startswith("{")][-1]
    b = json.loads(line)
    out["algorithmic_bytes_per_pair_pass"] = b["roofline"]["bytes_per_pair_pass"]
    out["bench_line"] = {"value": b["value"], "roofline": b["roofline"]}
    if "hbm_bytes_per_pair_pass" in out:
        out["traffic_over_algorithmic"] = out["hbm_bytes_per_pair_pass"] / out["algorithmic_bytes_per_pair_pass"]
except Exception as e:   # noqa: BLE001
    out["bench_line_error"] = str(e)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402  (the ICP source hash the bench line checks before it reports this profile's traffic)
out["icp_source_hash"] = bench.icp_source_hash()
print(json.dumps(out, indent=1))
