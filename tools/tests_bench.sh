#!/bin/bash
# GPU box: every -m gpu test, then one default bench line.  usage: tools/tests_bench.sh <tag>
set -o pipefail
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/tb_$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']; c=d.get('config5',{})
print('bench', round(d['value'],1), 'resident', round(d['value_hbm_resident_inputs'] or 0,1), 'frac', round(r['frac'],3), '| lone', round(r['isolated']['align_ms_per_pair'],3), '| config5', round(c.get('value',0),1), round((c.get('roofline') or {}).get('frac') or 0,3), '| config2', round(d['config2']['value'],1), 'config3', round(d['config3']['value'],1))"
