#!/bin/bash
# GPU box: kernel trace of the default bench command (2 steps) -> per-kernel duration / GPU area and busy summary.
# usage: tools/trace_area.sh <tag> [bench args]
R=$GRAFT_REPO_ROOT; TAG=${1:-ta}; shift; OUT=$R/gpurun_out/ta_$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-isolated "$@" > $OUT/bench.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 1; }
cd $R
T=$(ls $OUT/trace/*kernel_trace.csv | head -1)
python3 tools/kernel_area.py $T > $OUT/area.txt 2>&1
python3 tools/busy.py $T 1000 > $OUT/busy.txt 2>&1
rm -f $T
