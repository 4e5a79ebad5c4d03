#!/bin/bash
# Kernel-trace + PMC profiles of bench.py on the GPU box (run via gpurun from the repo root).
# usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r1}; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 4 --warmup 1 --no-cpu-baseline --no-resident $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc1 -o pmc1 -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc1.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $OUT/pmc2 -o pmc2 -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc2.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc3 -o pmc3 -- python3 $R/bench.py $ARGS > /dev/null 2> $OUT/pmc3.err || exit 4
echo profile-done
