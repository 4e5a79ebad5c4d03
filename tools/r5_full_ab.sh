#!/bin/bash
# GPU box: every -m gpu test on this tree, then two alternating default-bench A/B rounds against build/ab_base.
# usage: tools/r5_full_ab.sh <tag>
set -o pipefail
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/fab_$TAG; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/ab.sh ${TAG}a build/ab_base && bash tools/ab.sh ${TAG}b build/ab_base
