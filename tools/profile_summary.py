"""Summarise a tools/profile.sh output directory into profiles/<tag>/ (committed evidence):
  - kernel_stats.csv           rocprofv3 --kernel-trace --stats summary of the bench command
  - l0_pass.json               level-0 ICP pass: average duration (trace), FETCH_SIZE/WRITE_SIZE per launch
                               (separate --pmc passes), HBM bytes per launch with the gfx950 correction
usage: python tools/profile_summary.py gpurun_out/prof_<tag> profiles/<tag>
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

import numpy as np

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))[0]
shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
trace = glob.glob(os.path.join(src, "trace", "*kernel_trace.csv"))[0]
rows = list(csv.DictReader(open(trace)))


def is_l0(name):
    # the level-0 instantiation carries template tag TOP = 1: k_icp_pass<METHOD, PF, 1, OCC>
    return re.search(r"k_icp_pass<\d+, \d+, 1[,>]", name) is not None or re.search(r"k_icp_passILi\d+ELi\d+ELi1E", name) is not None


icp = [r for r in rows if is_l0(r["Kernel_Name"])]
gmax = max(int(r["Grid_Size_X"]) for r in icp)
l0 = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in icp]
l0_pairs = [int(r["Grid_Size_Y"]) for r in icp]   # blockIdx.y = pair: pairs per batched launch


def pmc(name):
    vals = []
    for f in glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if is_l0(r["Kernel_Name"]) and r["Counter_Name"] == name:
                vals.append(float(r["Counter_Value"]))
    return float(np.median(vals)) if vals else None


def pmc_per_job(name, waves_per_job):
    """median over level-0 dispatches of counter / jobs (a batched launch runs one pass per pair: jobs =
    SQ_WAVES of the same dispatch, collected in the same --pmc pass, / waves of one job's grid)"""
    vals = []
    for f in glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv")):
        per = {}
        for r in csv.DictReader(open(f)):
            if is_l0(r["Kernel_Name"]):
                per.setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
        for d in per.values():
            if name in d and d.get("SQ_WAVES"):
                vals.append(d[name] / (d["SQ_WAVES"] / waves_per_job))
    return float(np.median(vals)) if vals else None


fetch, write = pmc("FETCH_SIZE"), pmc("WRITE_SIZE")
# one job's grid: the level-0 launch's x extent in workgroups x waves per workgroup
waves_per_job = (gmax // 64) if gmax else None
fetch_j = pmc_per_job("FETCH_SIZE", waves_per_job) if waves_per_job else None
write_j = pmc_per_job("WRITE_SIZE", waves_per_job) if waves_per_job else None
out = {
    "kernel": "k_icp_pass<PHOTO_DEPTH> level 0", "grid_threads": gmax, "launches": len(l0),
    "avg_duration_us": float(np.mean(l0)), "median_duration_us": float(np.median(l0)),
    "avg_pairs_per_launch": float(np.mean(l0_pairs)),
    "FETCH_SIZE_kB_per_launch": fetch, "WRITE_SIZE_kB_per_launch": write,
    # MI355X_MICROARCH.md §HBM: FETCH_SIZE counts 64 B per 128-B request on gfx950 -> double it
    "hbm_bytes_per_launch": (2 * fetch * 1024 + write * 1024) if fetch is not None and write is not None else None,
    "note": "FETCH_SIZE doubled per the gfx950 correction; Infinity-Cache hits are counted by the counter",
    # per pair-pass (a batched launch runs one level-0 pass per pair): the figure bench.py scales by its own
    # pairs per launch
    "waves_per_job": waves_per_job, "FETCH_SIZE_kB_per_pair_pass": fetch_j, "WRITE_SIZE_kB_per_pair_pass": write_j,
    "hbm_bytes_per_pair_pass": (2 * fetch_j * 1024 + write_j * 1024) if fetch_j is not None and write_j is not None else None,
}
for k in ("SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE",
          "TCC_HIT_sum", "TCC_MISS_sum", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VMEM_RD"):
    v = pmc(k)
    if v is not None:
        out[k] = v   # median over dispatches of the raw counter (dispatches differ in pairs per launch)
    if k != "SQ_WAVES" and waves_per_job:
        vj = pmc_per_job(k, waves_per_job)   # per dispatch: counter / its own pairs, then the median
        if vj is not None:
            out[k + "_per_pair_pass"] = vj
# the traced command's own bench line: its in-kernel-span roofline against the trace's durations and pairs
try:
    line = [l for l in open(os.path.join(src, "trace.out")) if l.startswith("{")][-1]
    b = json.loads(line)["roofline"]
    B = b["bytes_per_pair_pass"]
    out["traced_line"] = {"avg_launch_ms": b["avg_launch_ms"], "pairs_per_launch": b["pairs_per_launch"],
                          "frac": b["frac"], "bytes_per_pair_pass": B}
    out["trace_frac"] = out["avg_pairs_per_launch"] * B / (out["avg_duration_us"] * 1e-6) / 1e9 / 8000.0
    out["trace_frac_over_line_frac"] = out["trace_frac"] / b["frac"]
except Exception as e:   # noqa: BLE001
    out["traced_line_error"] = str(e)
# the ICP sources this profile measured (bench.py reports the traffic only while they are unchanged)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
out["icp_source_hash"] = bench.icp_source_hash()
out["tag"] = os.path.basename(os.path.normpath(dst))
json.dump(out, open(os.path.join(dst, "l0_pass.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
