#!/bin/bash
# Round-3 profile of the BENCHMARKED configuration (run via gpurun from the repo root):
#   trace pass   rocprofv3 --kernel-trace --stats of the default bench command (8 pipelines x 3 in flight,
#                dense queue), python's faulthandler on so that a crash names the Python frame it hit
#   PMC passes   the same command, one --pmc group per run (MI355X_MICROARCH.md block limits)
#   HiRes PMC    config 5's dense workload (8 x 1280x960, 50 level-0 iterations): FETCH_SIZE / WRITE_SIZE
#                per pair-pass, the one size whose level-0 working set exceeds the Infinity Cache
#   bench lines  both commands without the profiler (in-kernel spans vs the trace's durations)
# usage: tools/prof_r3.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-r3}; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves $*"
HARGS="--workload dense --rows 960 --cols 1280 --iters0 50 --frames 33 --steps 1 --warmup 1 --no-cpu-baseline --no-resident --no-isolated --streams 8 --depth 2 --min-run 4"
step() {   # step <name> <timeout> <cmd...>: stops the script on the first failure
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] $name"
    timeout -k 10 $to "$@" > $OUT/$name.out 2> $OUT/$name.err
    local rc=$?
    if [ $rc != 0 ]; then echo "$name failed rc=$rc"; tail -c 3000 $OUT/$name.err; return $rc; fi
}
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 -X faulthandler $R/bench.py $ARGS &&
step pmc1 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc1 -o pmc1 -- python3 $R/bench.py $ARGS &&
step pmc2 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE SQ_WAVES -d $OUT/pmc2 -o pmc2 -- python3 $R/bench.py $ARGS &&
step pmc3 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_WAVES -d $OUT/pmc3 -o pmc3 -- python3 $R/bench.py $ARGS &&
step bench 300 python3 $R/bench.py $ARGS &&
step hires_pmc1 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE SQ_WAVES -d $OUT/hires/pmc1 -o pmc1 -- python3 $R/bench.py $HARGS &&
step hires_pmc2 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_WAVES -d $OUT/hires/pmc2 -o pmc2 -- python3 $R/bench.py $HARGS &&
step hires_pmc3 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/hires/pmc3 -o pmc3 -- python3 $R/bench.py $HARGS &&
step hires_bench 300 python3 $R/bench.py $HARGS
rc=$?
cd $R
python3 tools/profile_summary.py $OUT $OUT/summary > $OUT/summary.txt 2>&1
python3 tools/hires_summary.py $OUT/hires $OUT/hires_bench.out > $OUT/summary/hires_pmc.json 2>&1
T=$(ls $OUT/trace/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$T" ] && python3 tools/busy.py $T 1000 > $OUT/summary/busy.txt 2>&1
[ -n "$T" ] && python3 tools/kernel_area.py $T > $OUT/summary/area.txt 2>&1
find $OUT -name "*kernel_trace.csv" -delete; find $OUT -name "*counter_collection.csv" -delete
find $OUT -name "*.csv" -size +4M -delete
echo profile rc=$rc
exit $rc
