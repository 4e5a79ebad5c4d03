#!/bin/bash
# GPU box: the profile evidence of a round's bench line (run via gpurun from the repo root).
#   trace        rocprofv3 --kernel-trace --stats of the default sequence command (quick legs, 2 steps)
#   pmc1..3      the same command, one --pmc group per run (MI355X_MICROARCH.md block limits)
#   hires_pmc1-3 config 5's dense workload (8 x 1280x960, 50 level-0 iterations): FETCH_SIZE / WRITE_SIZE per
#                pair-pass (its level-0 working set exceeds the Infinity Cache) and the SQ counters
#   hires_bench  that command's bench line without the profiler
# Summaries (l0_pass.json, hires_pmc.json, kernel_stats.csv, busy.txt, dense_gaps.txt) go to gpurun_out/pmc_<tag>/summary;
# the raw CSVs are deleted (gpurun copies back at most 64 MiB).
# usage: tools/pmc_round.sh <tag>
set -o pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT/summary
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves"
HARGS="--workload dense --rows 960 --cols 1280 --iters0 50 --frames 33 --steps 1 --warmup 1 --no-cpu-baseline --no-resident --no-isolated --streams 8 --depth 2"
step() {   # step <name> <timeout> <cmd...>: stops the script on the first failure
    local name=$1 to=$2; shift 2
    echo "[$(date +%T)] $name"
    timeout -k 10 $to "$@" > $OUT/$name.out 2> $OUT/$name.err
    local rc=$?
    if [ $rc != 0 ]; then echo "$name failed rc=$rc"; tail -c 3000 $OUT/$name.err; return $rc; fi
}
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py $ARGS &&
step pmc1 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc1 -o pmc1 -- python3 $R/bench.py $ARGS &&
step pmc2 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE SQ_WAVES -d $OUT/pmc2 -o pmc2 -- python3 $R/bench.py $ARGS &&
step pmc3 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_WAVES -d $OUT/pmc3 -o pmc3 -- python3 $R/bench.py $ARGS &&
step hires_pmc1 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE SQ_WAVES -d $OUT/hires/pmc1 -o pmc1 -- python3 $R/bench.py $HARGS &&
step hires_pmc2 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_WAVES -d $OUT/hires/pmc2 -o pmc2 -- python3 $R/bench.py $HARGS &&
step hires_pmc3 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/hires/pmc3 -o pmc3 -- python3 $R/bench.py $HARGS &&
step hires_bench 300 python3 $R/bench.py $HARGS
rc=$?
cd $R
cp $OUT/trace.out $OUT/summary/trace_bench.json 2>/dev/null
python3 tools/profile_summary.py $OUT $OUT/summary > $OUT/summary/summary.txt 2>&1
python3 tools/hires_summary.py $OUT/hires $OUT/hires_bench.out > $OUT/summary/hires_pmc.json 2> $OUT/summary/hires_summary.err
T=$(ls $OUT/trace/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$T" ] && python3 tools/busy.py $T 1000 > $OUT/summary/busy.txt 2>&1
[ -n "$T" ] && python3 tools/dense_gaps.py $T > $OUT/summary/dense_gaps.txt 2>&1
find $OUT -name "*kernel_trace.csv" -delete; find $OUT -name "*counter_collection.csv" -delete
find $OUT -name "*.csv" -size +4M -delete
for f in $OUT/*.err; do tail -c 20000 $f > $f.tail && mv $f.tail $f; done
echo profile rc=$rc
exit $rc
