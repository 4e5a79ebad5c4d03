#!/bin/bash
# Bench variants on one GPU (gpurun).  usage: tools/bench_variants.sh <tag> "<name>:<bench args>" ...
set -o pipefail
O=gpurun_out/var_$1; shift; mkdir -p $O
run() { local n=$1; shift; timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-resident --steps 4 --warmup 1 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']; h=d.get('pipeline_host_ms_per_pair',{})
print('%-14s value %6.1f  P %2d  L0 %5.1f us  iso %5.1f  host ms/pair %s' % ('$n', d['value'], d['config']['pipelines_per_gpu'], r['avg_launch_ms']*1e3, r['isolated']['avg_launch_ms']*1e3, {k: round(v,2) for k,v in h.items()}))"; }
for spec in "$@"; do run ${spec%%:*} ${spec#*:} || exit 1; done
