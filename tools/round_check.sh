#!/bin/bash
# One GPU call for a round checkpoint (via gpurun): GPU tests, isolated plane-half trace, bench variants.
# usage: tools/round_check.sh <tag> "<name>:<bench args>" ...
set -o pipefail
TAG=${1:-rc}; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/tests_$TAG.log 2>&1 || { tail -30 $R/gpurun_out/tests_$TAG.log; exit 1; }
tail -2 $R/gpurun_out/tests_$TAG.log
bash $R/tools/iso_trace.sh $TAG || exit 2
cd $R && bash tools/variants_r2.sh var_$TAG "$@" || exit 3
