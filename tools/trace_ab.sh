#!/bin/bash
# Kernel traces of the default bench in two checkouts on one box, with GPU-busy / concurrency / per-queue summaries.
# usage: tools/trace_ab.sh <tag> <dir> <dir> ...
TAG=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tr_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for d in "$@"; do
  n=$(basename $d); [ "$d" = "." ] && n=this
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o trace -- python3 $R/$d/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves > $O/$n.json 2> $O/$n.err || { echo "$n trace failed"; tail -5 $O/$n.err; exit 3; }
  f=$(find $O/$n -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/busy.py $f 700 40 > $O/${n}_busy.txt && python3 $R/tools/queue_busy.py $f 700 > $O/${n}_queues.txt && python3 $R/tools/busy_split.py $f 700 k_pyramid k_icp_pass k_src > $O/${n}_split.txt && python3 $R/tools/kernel_area.py $f > $O/${n}_area.txt
  echo "== $n $(python3 -c "import json; print(round(json.load(open('$O/$n.json'))['value'],1))") pairs/s"; head -4 $O/${n}_busy.txt; cat $O/${n}_queues.txt
  rm -f $f
done
