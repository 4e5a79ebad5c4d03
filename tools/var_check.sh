#!/bin/bash
# GPU box: the dense-path and sequence GPU tests against an experiment variant library (extra environment in
# $TEST_ENV), then bench A/B of variants.
# usage: [TEST_ENV="K=V ..."] tools/var_check.sh <tag> <variant lib> "<name>|<dir>|<env>|<bench args>" ...
set -o pipefail
TAG=$1; LIB=$2; shift 2
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/vc_$TAG; mkdir -p $O
cd $R
env R360_LIB=$R/$LIB $TEST_ENV timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_sequence.py tests/test_gpu_batch_align.py tests/test_gpu_hires.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_mix.sh $TAG ${REPS:-2} "$@"
