#!/bin/bash
# GPU box: the default bench line under several environment settings (one line each, key numbers printed).
# usage: tools/bench_env.sh "<ENV=.. ENV2=..>" ...   ("-" = no extra environment); BARGS = extra bench args
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/benv
i=0
for e in "$@"; do
  i=$((i+1)); [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python3 $R/bench.py --steps 5 --no-cpu-baseline --no-config5 $BARGS > $R/gpurun_out/benv/b$i.json 2> $R/gpurun_out/benv/b$i.err || { echo "[$e] failed"; tail -3 $R/gpurun_out/benv/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$R/gpurun_out/benv/b$i.json')); r=d['roofline']; i=r['isolated']; print('[$e]', round(d['value'],1), 'pairs/s (resident', round(d['value_hbm_resident_inputs'] or 0,1), ') L0', round(r['avg_launch_ms']*1e3/r['pairs_per_launch'],2), 'us/pp at', round(r['pairs_per_launch'],2), 'frac', round(r['frac'],3), '| iso', round(i['avg_launch_ms']*1e3,2), 'us frac', round(i['frac'] or 0,3))"
done
