#!/bin/bash
# GPU box: dense-alone VGA bench line (level-0 in-kernel span per pair-pass) for experiment libraries
# (tools/exp_variants.sh).  usage: [PF=6] tools/exp_dense.sh <variant>[:<pf>] ...
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/exp
for vv in "$@"; do
  v=${vv%%:*}; pf=${vv#*:}; [ "$pf" = "$vv" ] && pf=${PF:-6}
  R360_LIB=$R/rgbd360_amd/lib/exp/lib_$v.so R360_ICP_PF=$pf timeout -k 10 200 python3 $R/bench.py --workload dense --steps 2 --warmup 1 \
    --no-cpu-baseline --no-resident --no-config5 --no-isolated > $R/gpurun_out/exp/dense_${v}_$pf.json 2> $R/gpurun_out/exp/dense_${v}_$pf.err \
    || { echo "$v failed"; tail -3 $R/gpurun_out/exp/dense_${v}_$pf.err; exit 1; }
  python3 -c "import json; d=json.load(open('$R/gpurun_out/exp/dense_${v}_$pf.json')); r=d['roofline']; print('$v PF $pf', round(d['value'],1), 'pairs/s; L0', round(r['avg_launch_ms']*1e3/r['pairs_per_launch'],2), 'us/pair-pass, frac', round(r['frac'],3))"
done
