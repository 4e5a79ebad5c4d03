#!/bin/bash
# GPU box, round checkpoint: every -m gpu test, smoke(), the default bench line (CPU leg, config-5 and halves legs,
# traffic from profiles/latest), then one rank's shard alone (--emulate 0/8 and 7/8) beside an N=1 line.
# usage: tools/close.sh <tag>   (results in gpurun_out/close_<tag>/)
set -o pipefail
TAG=${1:-r4}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/close_$TAG; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -3 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']; c=d.get('config5',{}); cr=c.get('roofline',{})
print('bench', round(d['value'],1), 'pairs/s, resident', round(d['value_hbm_resident_inputs'] or 0,1), 'frac', round(r['frac'],3), 'traffic', r['traffic'],
      '| lone', r['isolated']['align_ms_per_pair'], 'ms L0', round(r['isolated']['avg_launch_ms']*1e3,2), 'us | config5', round(c.get('value',0),1), 'frac', round(cr.get('frac',0) or 0,3), 'traffic', cr.get('traffic'),
      '| config2', (d.get('config2') or {}).get('value'), 'config3', (d.get('config3') or {}).get('value'), '| cpu', d.get('cpu_baseline',{}).get('value'), '| seq', (d.get('sequential_cpp') or {}).get('value'), '| c1', d.get('config1'), '| matcher', d.get('pbmap_matcher'))"
run() { local n=$1; shift; timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 4; }
  python3 -c "
import json; d=json.load(open('$O/$n.json')); r=d['roofline']
print('%-6s %7.1f pairs/s per GPU  P %2d  pairs %3d  L0 frac %.3f' % ('$n', d['value'], d['config']['pipelines_per_gpu'], d['config']['pairs_per_step_this_rank'], r['frac'] or 0))"; }
timeout -k 10 200 ./build/bin/OdometryRGBD360 --throughput 256 3 > $O/cpp_throughput.txt 2>&1 && cat $O/cpp_throughput.txt && run n1 && run s0of8 --emulate 0/8 && run s7of8 --emulate 7/8
