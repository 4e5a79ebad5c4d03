#!/bin/bash
# GPU box: the sequence GPU tests, then N=1 and emulated 1/8 shards (one rank's pairs alone on one GPU).
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/sh_$TAG; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_sequence.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { local n=$1; shift; timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves --steps 5 --warmup 1 "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 4; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']; h=d['pipeline_host_ms_per_pair']
print('%-6s %7.1f pairs/s per GPU  P %2d  pairs %3d  L0 frac %.3f  build_enqueue %.2f ms  wait_pbmaps %.2f' % ('$n', d['value'], d['config']['pipelines_per_gpu'], d['config']['pairs_per_step_this_rank'], r['frac'] or 0, h['load_split']['build_enqueue'], h['pbmap_stage_split']['wait_frame_pbmaps']))"; }
run n1 "$@" && run s0of8 --emulate 0/8 "$@" && run s7of8 --emulate 7/8 "$@" && run s3of8 --emulate 3/8 "$@"
