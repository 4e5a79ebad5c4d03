#!/bin/bash
# GPU box, one round-4 iteration: every -m gpu test, GN-step stamps (stamps build: make -C rgbd360_amd/csrc stamps)
# and the lone pair, then a bench line without the CPU leg (config-5 leg included).
# usage: tools/r4_iter.sh <tag> [--no-tests] [extra bench args]
set -o pipefail
TAG=${1:-a}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/it4_$TAG; mkdir -p $O; cd $R
if [ "$1" == "--no-tests" ]; then shift; else
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
if [ -f rgbd360_amd/lib/librgbd360_hip_stamps.so ]; then
  R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_stamps.so ALIGN=1 R360_DIAG_EXTRA_ITERS=1 timeout -k 10 120 python3 tools/stamps.py > $O/stamps_cont.txt 2>&1 || { tail $O/stamps_cont.txt; exit 2; }
  grep -E "align last|eval at" $O/stamps_cont.txt
fi
timeout -k 10 120 python3 tools/lone_align.py 30 > $O/lone.txt 2>&1 || { tail $O/lone.txt; exit 3; }
tail -2 $O/lone.txt
timeout -k 10 400 python3 bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 4; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']; c=d.get('config5',{}); iso=r.get('isolated') or {}
print('bench', round(d['value'],1), 'pairs/s, resident', round(d.get('value_hbm_resident_inputs') or 0,1), 'frac', round(r['frac'],3),
      '| lone L0', round((iso.get('avg_launch_ms') or 0)*1e3,2), 'us, align', iso.get('align_ms_per_pair'), 'ms | config5', round(c.get('value',0),1),
      'pairs/s frac', round((c.get('roofline') or {}).get('frac',0) or 0,3))"
