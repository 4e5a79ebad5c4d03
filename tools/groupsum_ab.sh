#!/bin/bash
# GPU box: two-level record sum (shipped default) vs the flat sum (librgbd360_hip_flat.so): per-level stamps,
# lone-pair alignFrames360, the -m gpu tests and two short default-bench lines each.
# usage: tools/groupsum_ab.sh <tag>     (results in gpurun_out/gsum_<tag>/)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/gsum_${1:-ab}; mkdir -p $O; cd $R
L=$R/rgbd360_amd/lib
R360_LIB=$L/librgbd360_hip_stamps.so NB=512 timeout -k 10 120 python3 -u tools/stamps.py > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
head -5 $O/stamps.txt
for v in "" _flat "" _flat; do
  R360_LIB=$L/librgbd360_hip$v.so timeout -k 10 120 python3 -u tools/lone_align.py 30 >> $O/lone.txt 2>&1 || { tail $O/lone.txt; exit 2; }
done
cat $O/lone.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 3; }
tail -1 $O/gpu_tests.log
i=0
for v in "" _flat "" _flat; do
  i=$((i+1))
  R360_LIB=$L/librgbd360_hip$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-resident --no-config5 --steps 5 --warmup 1 > $O/bench${v}_$i.json 2> $O/bench${v}_$i.err || { tail $O/bench${v}_$i.err; exit 4; }
  python3 -c "import json; d=json.load(open('$O/bench${v}_$i.json')); r=d['roofline']; print('lib$v', round(d['value'],1), 'pairs/s  L0', round(r['avg_launch_ms']*1e3,2), 'us frac', round(r['frac'],3), ' lone L0', round(r['isolated']['avg_launch_ms']*1e3,2), 'us align', round(r['isolated']['align_ms_per_pair'],3), 'ms')"
done
