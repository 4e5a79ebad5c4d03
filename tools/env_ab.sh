#!/bin/bash
# GPU box: default bench lines (headline only, 10 steps) on the experiment library under several environments,
# each run twice in alternation.  usage: tools/env_ab.sh <tag> "<name>|<env>" ...  (results in gpurun_out/envab_<tag>/)
set -o pipefail
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/envab_$TAG; mkdir -p $O; cd $R
B="--no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves ${EXTRA:-}"
for rep in 1 2; do
  for v in "$@"; do
    IFS='|' read -r n e <<< "$v"
    env R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_exp.so $e timeout -k 10 200 python3 -u bench.py $B > $O/${n}_$rep.json 2> $O/${n}_$rep.err || { echo "$n failed"; tail -5 $O/${n}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${n}_$rep.json'))
print('%-10s rep $rep %8.1f pairs/s' % ('$n', d['value']))"
  done
done
