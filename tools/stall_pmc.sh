#!/bin/bash
# GPU box: stall-attribution counters of the level-0 ICP pass in the dense-alone VGA bench (PF from the env).
# usage: [R360_ICP_PF=6] tools/stall_pmc.sh <tag>
export R360_LIB=${R360_LIB:-${GRAFT_REPO_ROOT:-.}/rgbd360_amd/lib/librgbd360_hip_exp.so}   # knobs: experiment build (make -C rgbd360_amd/csrc exp)
R=$GRAFT_REPO_ROOT; TAG=${1:-st}; OUT=$R/gpurun_out/stall_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
DARGS="--workload dense --steps 1 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-isolated"
timeout -k 10 200 python3 $R/bench.py $DARGS > $OUT/dense.json 2> $OUT/dense.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU -d $OUT/pmc1 -o p -- python3 $R/bench.py $DARGS > /dev/null 2> $OUT/p1.err || { tail -3 $OUT/p1.err; exit 2; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_SMEM -d $OUT/pmc2 -o p -- python3 $R/bench.py $DARGS > /dev/null 2> $OUT/p2.err || { tail -3 $OUT/p2.err; exit 3; }
python3 $R/tools/hires_summary.py $OUT $OUT/dense.json > $OUT/summary.json 2>&1
python3 - $OUT <<'PY'
import csv, glob, json, re, sys, numpy as np
out = sys.argv[1]
def is_l0(n): return re.search(r"k_icp_passILi\d+ELi\d+ELi1E", n) or re.search(r"k_icp_pass<\d+, \d+, 1[,>]", n)
per = {}
for d in glob.glob(out + "/pmc*"):
    jobs = {}
    for f in glob.glob(d + "/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if is_l0(r["Kernel_Name"]): jobs[r["Dispatch_Id"]] = (int(r["Grid_Size_Y"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for f in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if is_l0(r["Kernel_Name"]) and r["Dispatch_Id"] in jobs:
                per.setdefault(r["Counter_Name"], []).append((float(r["Counter_Value"]), *jobs[r["Dispatch_Id"]]))
res = {}
for k, v in per.items():
    res[k + "_per_pair"] = float(np.median([c / j for c, j, _ in v]))
    res[k + "_per_us"] = float(np.median([c / t for c, _, t in v]))
print(json.dumps(res, indent=1))
PY
find $OUT -name "*.csv" -delete
