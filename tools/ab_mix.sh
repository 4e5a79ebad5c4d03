#!/bin/bash
# Bench variants by environment AND arguments, alternating, on one box.
# usage: tools/ab_mix.sh <tag> <reps> "<name>|<dir>|<env>|<bench args>" ...
set -o pipefail
TAG=$1; REPS=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/abm_$TAG; mkdir -p $O
one() { local name=$1 dir=$2 envs=$3 a=$4
  (cd $R/$dir && env $envs timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-resident --no-config5 ${ISO:+--no-isolated} --no-halves --steps 10 --warmup 2 $a > $O/$name.json 2> $O/$name.err) || { echo "$name failed"; tail -5 $O/$name.err; exit 4; }
  python3 -c "
import json; d=json.load(open('$O/$name.json')); r=d['roofline']; h=d['pipeline_host_ms_per_pair']
ppl = r.get('pairs_per_launch') or 0; l0 = r['avg_launch_ms']*1e3/ppl if ppl else 0.0
print('%-12s lone %s %7.1f pairs/s  L0 %.1f us/pair  batch %.2f  wait_pbmaps %.2f  dense_wait %.2f  load %.2f ms' % ('$name', (r.get('isolated') or {}).get('align_ms_per_pair'), d['value'], l0, ppl, h['pbmap_stage_split']['wait_frame_pbmaps'], h['dense_wait'], h['load_build_enqueue']), {k: round(v, 2) for k, v in h.get('load_split', {}).items()}, d.get('plane_queue'))"; }
for rep in $(seq 1 $REPS); do for v in "$@"; do IFS='|' read -r n d e a <<< "$v"; one ${n}_$rep "$d" "$e" "$a" || exit 4; done; done
