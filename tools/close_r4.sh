#!/bin/bash
# GPU box: the round-end checks in one call — every -m gpu test, smoke(), the default bench line (CPU baseline and
# config-5 leg included), then the profile of the benchmarked configuration (tools/prof_r3.sh).
# usage: tools/close_r4.sh <tag>     (results in gpurun_out/close_<tag>/ and gpurun_out/prof_<tag>/)
set -o pipefail
TAG=${1:-r3}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/close_$TAG; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; c=d.get('config5',{}); print('bench', round(d['value'],1), 'pairs/s, resident', round(d['value_hbm_resident_inputs'] or 0,1), 'frac', round(r['frac'],3), 'traffic', r['traffic'], '| lone L0', round(r['isolated']['avg_launch_ms']*1e3,2), 'us | config5', round(c.get('value',0),1), 'pairs/s frac', round(c.get('roofline',{}).get('frac',0) or 0,3), '| cpu', d.get('cpu_baseline',{}).get('value'))"
bash tools/prof_r3.sh $TAG
