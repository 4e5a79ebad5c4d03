#!/bin/bash
# GPU box: short bench lines of pipeline variants, one after another in one session (tools/r4_var.sh <tag> "<args>"...)
set -o pipefail
TAG=${1:-v}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/var_$TAG; mkdir -p $O; cd $R
i=0
for a in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves $a > $O/v$i.json 2> $O/v$i.err || { tail -5 $O/v$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/v$i.json')); h=d['pipeline_host_ms_per_pair']; print('[$a]', round(d['value'],1), 'pairs/s frac', round(d['roofline']['frac'],3), 'ppl', round(d['roofline']['pairs_per_launch'],1), 'wait_pbmap', round(h['pbmap_stage_split']['wait_frame_pbmaps'],2), 'dense_wait', round(h['dense_wait'],2))"
  i=$((i+1))
done
