#!/bin/bash
# GPU box: short default bench lines on the experiment build under grid knobs (R360_ICP_PXT, R360_ICP_CAP), one after
# another in one session.  usage: tools/r4_knobs.sh <tag> "<ENV=V ...>"...   ("" = the experiment build's defaults)
set -o pipefail
TAG=${1:-k}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/knob_$TAG; mkdir -p $O; cd $R
export R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_exp.so
i=0
for e in "$@"; do
  env $e timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-halves > $O/k$i.json 2> $O/k$i.err || { tail -5 $O/k$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/k$i.json')); r=d['roofline']; iso=r['isolated']; print('[$e]', round(d['value'],1), 'pairs/s frac', round(r['frac'],3), 'ppl', round(r['pairs_per_launch'],1), '| lone', round(iso['align_ms_per_pair'],3), 'ms L0', round(iso['avg_launch_ms']*1e3,1), 'us')"
  i=$((i+1))
done
