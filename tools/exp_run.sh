#!/bin/bash
# GPU box: kernel-trace durations of the level-0 ICP pass for experiment libraries (tools/exp_variants.sh).
# usage: tools/exp_run.sh <variant> ...     (env LEVELS, default 0)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  OUT=$R/gpurun_out/exp_$v
  rm -rf $OUT; mkdir -p $OUT
  R360_LIB=$R/rgbd360_amd/lib/exp/lib_$v.so LEVELS=${LEVELS:-0} timeout -k 10 120 rocprofv3 --kernel-trace --stats \
     --output-format csv -d $OUT -o t -- python3 $R/tools/icp_bench.py 30 > $OUT/out.txt 2>&1 || { echo "$v failed"; exit 1; }
  python3 - "$OUT" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_icp_pass" in r["Name"]:
        print(f"{sys.argv[2]:10s} {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.2f} us  min {float(r['MinNs'])/1e3:8.2f}")
PY
  grep "level" $OUT/out.txt | sed "s/^/$v  events: /"
done
