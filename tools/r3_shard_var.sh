#!/bin/bash
# GPU box: the emulated 1/8 shards under pipeline-sizing variants.  usage: tools/r3_shard_var.sh <tag> "<name>:<args>" ...
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/shv_${1:-x}; shift; mkdir -p $O
for spec in "$@"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-resident --no-config5 --no-isolated --steps 5 --warmup 1 $a > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('%-12s %7.1f pairs/s per GPU  P %2d  pairs %3d  L0 frac %.3f  batch %.2f' % ('$n', d['value'], d['config']['pipelines_per_gpu'], d['config']['pairs_per_step_this_rank'], r['frac'] or 0, r['pairs_per_launch']))"
done
