#!/bin/bash
# Bench variants by environment (experiment library knobs), alternating, on one box.
# usage: tools/ab_env.sh <tag> "<name>|<dir>|<env assignments>" ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/abe_$TAG; mkdir -p $O
one() { local name=$1 dir=$2 envs=$3
  (cd $R/$dir && env $envs timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves --steps 10 --warmup 2 > $O/$name.json 2> $O/$name.err) || { echo "$name failed"; tail -5 $O/$name.err; exit 4; }
  python3 -c "
import json; d=json.load(open('$O/$name.json')); r=d['roofline']; h=d['pipeline_host_ms_per_pair']
print('%-14s %7.1f pairs/s  L0 %.1f us/pair  batch %.2f  wait_pbmaps %.2f ms' % ('$name', d['value'], r['avg_launch_ms']*1e3/r['pairs_per_launch'], r['pairs_per_launch'], h['pbmap_stage_split']['wait_frame_pbmaps']))"; }
for rep in 1 2; do for v in "$@"; do IFS='|' read -r n d e <<< "$v"; one ${n}_$rep $d "$e" || exit 4; done; done
