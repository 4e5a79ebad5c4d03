#!/bin/bash
# GPU box: one rank's shard alone (--emulate r/8) beside N=1, at the bench's default steps (10) and warmup (2).
# usage: tools/shard10.sh <tag>   (results in gpurun_out/sh10_<tag>/)
set -o pipefail
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/sh10_$TAG; mkdir -p $O; cd $R
run() { local n=$1; shift; timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 4; }
  python3 -c "
import json; d=json.load(open('$O/$n.json'))
print('%-6s %7.1f pairs/s per GPU  steps %d  pairs %3d  ms/step %.2f  extra builds/step %s' % ('$n', d['value'], d['steps'], d['config']['pairs_per_step_this_rank'], d['ms_per_step'], d['config'].get('extra_frame_builds_per_step')))"; }
run n1 && run s0 --emulate 0/8 && run s7 --emulate 7/8 && run s3 --emulate 3/8 && run n1b && run s7b --emulate 7/8
