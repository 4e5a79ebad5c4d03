#!/bin/bash
# GPU box: every -m gpu test, then tools/lone_align.py on the product library.
# usage: tools/r5_quick.sh <tag>   (results in gpurun_out/quick_<tag>/)
set -o pipefail
TAG=${1:-q}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/quick_$TAG; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python3 -u tools/lone_align.py 30 > $O/lone.txt 2>&1 || { tail -5 $O/lone.txt; exit 2; }
cat $O/lone.txt
