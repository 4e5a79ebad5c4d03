#!/bin/bash
# GPU box: the -m gpu suite, then bench variants (tools/ab_mix.sh syntax).
# usage: tools/r5_iter.sh <tag> "<name>|<dir>|<env>|<bench args>" ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/it_$TAG; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/ab_mix.sh $TAG 1 "$@"
