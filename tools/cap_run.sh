#!/bin/bash
# GPU box: kernel-trace duration of the level-0 ICP pass (eval mode, tools/icp_bench.py) per grid cap.
# usage: CAPS="512 1024" tools/cap_run.sh
export R360_LIB=${R360_LIB:-${GRAFT_REPO_ROOT:-.}/rgbd360_amd/lib/librgbd360_hip_exp.so}   # knobs: experiment build (make -C rgbd360_amd/csrc exp)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for cap in ${CAPS:-512 768 1024 1536 2048}; do
  OUT=$R/gpurun_out/cap_$cap
  rm -rf $OUT; mkdir -p $OUT
  R360_ICP_CAP=$cap LEVELS=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o t \
     -- python3 $R/tools/icp_bench.py 30 > $OUT/out.txt 2>&1 || { echo "cap $cap failed"; exit 1; }
  python3 - "$OUT" "$cap" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_icp_pass<2, 3, 1" in r["Name"]:
        print(f"cap {sys.argv[2]:>5s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.2f} us  min {float(r['MinNs'])/1e3:8.2f}")
PY
done
