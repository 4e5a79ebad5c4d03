#!/bin/bash
# GPU box: config 5's dense workload (8 x 1280x960, 50 level-0 iterations) by environment / extra bench args.
# usage: tools/hires_sweep.sh <tag> "<name>|<env>|<args>" ...   (results in gpurun_out/hs_<tag>/)
set -o pipefail
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/hs_$TAG; mkdir -p $O; cd $R
H="--workload dense --rows 960 --cols 1280 --iters0 50 --frames 33 --steps 2 --warmup 1 --no-cpu-baseline --no-resident --no-isolated --no-config5 --no-halves --streams 8 --depth 2 --min-run 4"
for v in "$@"; do
  IFS='|' read -r n e a <<< "$v"
  env $e timeout -k 10 200 python3 -u bench.py $H $a > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('%-12s %7.1f pairs/s  frac %.3f  L0 %.1f us/launch  %.2f pairs/launch' % ('$n', d['value'], r['frac'] or 0, r['avg_launch_ms']*1e3, r['pairs_per_launch']))"
done
