#!/bin/bash
# A/B of the default bench line between this tree and another checkout (build/ab_*), alternating, on one box.
# usage: tools/ab.sh <tag> <other-checkout-dir> [bench args]
set -o pipefail
TAG=$1; OTHER=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_$TAG; mkdir -p $O
one() { local name=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves --steps 10 --warmup 2 "$@" > $O/$name.json 2> $O/$name.err) || { echo "$name failed"; tail -5 $O/$name.err; exit 4; }
  python3 -c "
import json; d=json.load(open('$O/$name.json')); r=d['roofline']; h=d['pipeline_host_ms_per_pair']
print('%-8s %7.1f pairs/s  L0 %.1f us/pair  batch %.2f  wait_pbmaps %.2f ms' % ('$name', d['value'], r['avg_launch_ms']*1e3/r['pairs_per_launch'], r['pairs_per_launch'], h['pbmap_stage_split']['wait_frame_pbmaps']))"; }
one new1 $R "$@" && one old1 $R/$OTHER "$@" && one new2 $R "$@" && one old2 $R/$OTHER "$@"
