#!/bin/bash
# GPU box: kernel trace of the default bench command (no extra legs), its dense-stream gaps and busy summary.
# usage: tools/r5_trace.sh <tag>   (results in gpurun_out/trace_<tag>/)
set -o pipefail
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/trace_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cd $R
T=$(ls $O/trace/*kernel_trace.csv | head -1); S=$(ls $O/trace/*kernel_stats.csv | head -1)
cp $S $O/kernel_stats.csv
python3 tools/dense_gaps.py $T > $O/dense_gaps.txt 2>&1; cat $O/dense_gaps.txt
python3 tools/busy.py $T 1000 > $O/busy.txt 2>&1; head -3 $O/busy.txt
python3 tools/kernel_area.py $T > $O/area.txt 2>&1 || true
python3 -c "import json; d=json.load(open('$O/bench.json')); print('traced bench', round(d['value'],1), d['config']['gpu_max_hw_queues'])"
find $O -name "*.csv" -size +4M -delete
