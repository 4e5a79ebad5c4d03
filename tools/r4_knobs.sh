#!/bin/bash
# GPU box: short default bench lines (no CPU leg, no config-5 / halves legs) under library builds and knobs, one after
# another in one session.  usage: tools/r4_knobs.sh <tag> "[<lib-suffix>:]<ENV=V ...>"...
#   lib-suffix: rgbd360_amd/lib/librgbd360_hip_<suffix>.so (default exp, the experiment build); "product:" = the
#   shipped library.  "" = the experiment build's defaults.
set -o pipefail
TAG=${1:-k}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/knob_$TAG; mkdir -p $O; cd $R
i=0
for spec in "$@"; do
  suf=exp; e=$spec
  case "$spec" in *:*) suf=${spec%%:*}; e=${spec#*:};; esac
  if [ "$suf" == "product" ]; then lib=$R/rgbd360_amd/lib/librgbd360_hip.so; else lib=$R/rgbd360_amd/lib/librgbd360_hip_$suf.so; fi
  env R360_LIB=$lib $e timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-halves > $O/k$i.json 2> $O/k$i.err || { tail -5 $O/k$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/k$i.json')); r=d['roofline']; iso=r['isolated']; print('[$spec]', round(d['value'],1), 'pairs/s frac', round(r['frac'],3), 'ppl', round(r['pairs_per_launch'],1), 'L0', round(r['avg_launch_ms']*1e3,1), 'us | lone', round(iso['align_ms_per_pair'],3), 'ms L0', round(iso['avg_launch_ms']*1e3,1), 'us')"
  i=$((i+1))
done
