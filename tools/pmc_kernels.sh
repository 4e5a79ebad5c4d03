#!/bin/bash
# One rocprofv3 --pmc pass over a short bench run, summarised per kernel (tools/pmc_kernels.py).
# usage (via gpurun): tools/pmc_kernels.sh <tag> [bench args]
set -o pipefail
TAG=${1:-k}; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmck_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU -d $OUT/pmc -o pmc -- python3 $R/bench.py --streams 4 --steps 1 --warmup 1 --frames 64 --no-cpu-baseline --no-resident "$@" > $OUT/bench.json 2> $OUT/pmc.err || { tail -c 3000 $OUT/pmc.err; exit 1; }
cd $R
python3 tools/pmc_kernels.py $OUT/pmc 45 > $OUT/kernels.txt 2>&1
find $OUT -name "*.csv" -delete
tail -c 20000 $OUT/pmc.err > $OUT/t && mv $OUT/t $OUT/pmc.err
cat $OUT/kernels.txt
