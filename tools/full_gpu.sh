#!/bin/bash
# GPU box: the whole -m gpu suite without stopping at the first failure, the synthetic odometry app's poses and the
# lone-pair timing of the product library.  usage: tools/full_gpu.sh <tag>  (results in gpurun_out/full_<tag>/)
set -o pipefail
TAG=${1:-x}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/full_$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "^FAILED|passed|failed" $O/gpu_tests.log | tail -25
[ $rc -le 1 ] || exit $rc
timeout -k 10 100 ./build/bin/OdometryRGBD360 --synthetic 6 > $O/odo.txt 2>&1 && grep pose $O/odo.txt &&
timeout -k 10 120 python3 -u tools/lone_align.py 30 > $O/lone.txt 2>&1 && cat $O/lone.txt
