#!/bin/bash
# GPU box: one rank's shard alone (--emulate r/8) at several pipeline counts (--streams), beside N=1 lines.
# usage: tools/shard_p.sh <tag> "<streams...>"   (results in gpurun_out/shp_<tag>/)
set -o pipefail
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/shp_$TAG; mkdir -p $O; cd $R
run() { local n=$1; shift; timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves --steps 5 --warmup 1 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 4; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('%-10s %7.1f pairs/s per GPU  P %2d  pairs %3d  ms/step %.2f' % ('$n', d['value'], d['config']['pipelines_per_gpu'], d['config']['pairs_per_step_this_rank'], d['ms_per_step']))"; }
for p in $2; do run s7_p$p --emulate 7/8 --streams $p && run s0_p$p --emulate 0/8 --streams $p || exit 4; done
run n1_p12 --streams 12
