#!/bin/bash
# VALU instructions per pixel of the level-0 ICP pass (eval mode) for the current build.
# usage (GPU box): [PMC="counters"] tools/icp_pmc.sh <tag> [env assignments...]
set -o pipefail
TAG=${1:-x}; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/icp_pmc_$TAG
mkdir -p $OUT
env "$@" LEVELS=0 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv --pmc ${PMC:-SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD} -d $OUT -o pmc -- python3 $R/tools/icp_bench.py 20 > $OUT/out.txt 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/*counter_collection.csv")[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "k_icp_pass" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
px = 640 * 3840
for k, v in agg.items():
    v = sorted(v)[len(v) // 2]
    print(f"{k:22s} median {v:14.0f}   per pixel {v * 64 / px if 'INSTS' in k else v / px:9.3f}")
PY
grep "level 0" $OUT/out.txt
