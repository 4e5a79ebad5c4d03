#!/bin/bash
# GPU box: the default bench line at N=1 next to one rank's shard alone (--emulate r/N: that rank's pairs, halo
# frames and pipelines, on one GPU) and the N=1 line with HIP's default 4 hardware queues.
# usage: tools/r3_shards.sh <tag>   (results in gpurun_out/sh_<tag>/)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/sh_${1:-x}; mkdir -p $O
run() { local n=$1; shift; env $E timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-resident --no-config5 --no-isolated --steps 5 --warmup 1 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('%-10s %7.1f pairs/s per GPU  P %2d  pairs %3d  L0 frac %.3f' % ('$n', d['value'], d['config']['pipelines_per_gpu'], d['config']['pairs_per_step_this_rank'], r['frac'] or 0))"; }
E="" run n1 && E="" run s0of2 --emulate 0/2 && E="" run s0of4 --emulate 0/4 && E="" run s0of8 --emulate 0/8 && \
E="" run s7of8 --emulate 7/8 && E="GPU_MAX_HW_QUEUES=4" run hwq4 && E="" run n1b
