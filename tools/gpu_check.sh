#!/bin/bash
# GPU round trip used during development: gpu tests + a kernel-traced bench (run via gpurun).
# usage: tools/gpu_check.sh <tag> [bench args]
TAG=${1:-x}; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 480 python -m pytest $R/tests -m gpu -q > $R/gpurun_out/tests_$TAG.log 2>&1
echo "pytest exit $?" >> $R/gpurun_out/tests_$TAG.log
tail -3 $R/gpurun_out/tests_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o trace -- python3 $R/bench.py --steps 10 --warmup 2 "$@" > $R/gpurun_out/bench_$TAG.json 2>&1
echo "bench exit $?"
grep '^{' $R/gpurun_out/bench_$TAG.json | cut -c1-400
