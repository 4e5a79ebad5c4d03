#!/bin/bash
# Kernel-trace + PMC profiles of bench.py on the GPU box (run via gpurun from the repo root).
# usage: tools/profile.sh <tag> [bench args...]
#   trace pass: rocprofv3 --kernel-trace --stats of `bench.py --streams 4` (and the same command's own bench
#     line), because rocprofv3 7.2's dispatch hook crashes (SIGSEGV in the launch path, 8 of 8 attempts) when
#     16 host threads launch concurrently (the default --streams 16); 1 or 4 threads trace cleanly
#   PMC passes: the default command (counters are collected per dispatch, kernels serialised)
# The raw CSVs are summarised on the box (tools/profile_summary.py, tools/busy.py) and deleted: gpurun
# copies back at most 64 MiB.
set -o pipefail
TAG=${1:-r1}; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-resident $*"
TARGS="--streams 4 $ARGS"
rc=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py $TARGS > $OUT/trace_bench.json 2> $OUT/trace.err || rc=1
[ $rc = 0 ] && { timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc1 -o pmc1 -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc1.err || rc=2; }
[ $rc = 0 ] && { timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE SQ_WAVES -d $OUT/pmc2 -o pmc2 -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc2.err || rc=3; }
[ $rc = 0 ] && { timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_WAVES -d $OUT/pmc3 -o pmc3 -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc3.err || rc=4; }
# the traced command's bench line without the profiler (its in-kernel spans vs the trace's durations)
[ $rc = 0 ] && { timeout -k 10 300 python3 $R/bench.py $TARGS > $OUT/bench_streams4.json 2> $OUT/bench_streams4.err || rc=5; }
cd $R
python3 tools/profile_summary.py $OUT $OUT/summary > $OUT/summary.txt 2>&1
T=$(ls $OUT/trace/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$T" ] && python3 tools/busy.py $T 1000 > $OUT/summary/busy.txt 2>&1
find $OUT -name "*kernel_trace.csv" -delete; find $OUT -name "*counter_collection.csv" -delete
find $OUT -name "*.csv" -size +4M -delete
# keep only the tails of the error logs (a crash dumps long stacks)
for f in $OUT/*.err; do tail -c 20000 $f > $f.tail && mv $f.tail $f; done
echo profile rc=$rc
exit $rc
