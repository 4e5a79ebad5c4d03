#!/bin/bash
# GPU box: level-0 pass counters, dense half alone (VGA, batches of up to 16 pairs): SQ_INSTS_VALU and wave cycles per
# pair-pass, then FETCH_SIZE / WRITE_SIZE, plus the dense-alone bench line.  usage: tools/r4_pmc.sh <tag>
set -o pipefail
TAG=${1:-a}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc4_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--workload dense --steps 2 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves"
timeout -k 10 200 python3 $R/bench.py $A > $O/dense.json 2> $O/dense.err || { tail -5 $O/dense.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/p1 -o p -- python3 $R/bench.py $A > /dev/null 2> $O/p1.err || { tail -5 $O/p1.err; exit 2; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE SQ_WAVES -d $O/p2 -o p -- python3 $R/bench.py $A > /dev/null 2> $O/p2.err || { tail -5 $O/p2.err; exit 3; }
cd $R
python3 tools/pmc_l0.py $O > $O/summary.txt 2>&1; cat $O/summary.txt
find $O -name "*.csv" -size +2M -delete
