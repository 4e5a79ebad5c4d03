#!/bin/bash
# Isolated per-kernel durations: rocprofv3 kernel trace of one pipeline (--streams 1, no dense queue), so no
# kernel shares the GPU with another pipeline's.  usage (via gpurun): tools/iso_trace.sh <tag> [bench args]
set -o pipefail
TAG=${1:-iso}; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/iso_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --streams 1 --queue 0 --steps 1 --warmup 1 --frames 64 --no-cpu-baseline --no-resident --no-config5 "$@" > $OUT/bench.json 2> $OUT/trace.err || exit 1
cd $R
T=$(ls $OUT/trace/*kernel_trace.csv | head -1)
python3 tools/busy.py $T 100000 80 > $OUT/busy.txt 2>&1
python3 tools/plane_half_sum.py $OUT/busy.txt > $OUT/plane_half.txt 2>&1
python3 tools/kernel_area.py $T > $OUT/area.txt 2>&1
rm -f $T
tail -c 20000 $OUT/trace.err > $OUT/t && mv $OUT/t $OUT/trace.err
head -12 $OUT/plane_half.txt
