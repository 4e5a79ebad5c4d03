#!/bin/bash
# One GPU iteration (run through gpurun from the repo root): parity tests of the given files, the ICP pass
# micro-benchmark at levels 0-2 (eval mode, identity and true-motion poses) and the default bench line.
#   usage: tools/gpu_iter.sh <tag> [test files...]
set -o pipefail
TAG=${1:-it}; shift
O=gpurun_out/$TAG; mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
timeout -k 10 180 python -u tools/icp_bench.py 30 > $O/icp_bench.txt 2>&1 || { echo "icp_bench failed"; tail $O/icp_bench.txt; exit 2; }
POSE=path timeout -k 10 180 python -u tools/icp_bench.py 30 >> $O/icp_bench.txt 2>&1 || { echo "icp_bench path failed"; exit 3; }
cat $O/icp_bench.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 4; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value', round(d['value'],1), 'resident', round(d['value_hbm_resident_inputs'] or 0,1), 'L0 pipeline us', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],3), 'isolated us', round(r['isolated']['avg_launch_ms']*1e3,1), 'frac', round(r['isolated']['frac'],3))"
