#!/bin/bash
# GPU box: single-lane GN rank test + solve (shipped default) vs the wave-parallel forms (librgbd360_hip_gnwave.so):
# lone-pair alignFrames360, the -m gpu tests and short default-bench lines.  usage: tools/gn_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/gn_${1:-ab}; mkdir -p $O; cd $R
L=$R/rgbd360_amd/lib
for v in "" _gnwave "" _gnwave; do
  R360_LIB=$L/librgbd360_hip$v.so timeout -k 10 120 python3 -u tools/lone_align.py 30 >> $O/lone.txt 2>&1 || { tail $O/lone.txt; exit 2; }
done
cat $O/lone.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 3; }
tail -1 $O/gpu_tests.log
i=0
for v in "" _gnwave; do
  i=$((i+1))
  R360_LIB=$L/librgbd360_hip$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-resident --no-config5 --steps 5 --warmup 1 > $O/bench${v}_$i.json 2> $O/bench${v}_$i.err || { tail $O/bench${v}_$i.err; exit 4; }
  python3 -c "import json; d=json.load(open('$O/bench${v}_$i.json')); r=d['roofline']; print('lib$v', round(d['value'],1), 'pairs/s  L0', round(r['avg_launch_ms']*1e3,2), 'us frac', round(r['frac'],3), ' lone L0', round(r['isolated']['avg_launch_ms']*1e3,2), 'us align', round(r['isolated']['align_ms_per_pair'],3), 'ms')"
done
