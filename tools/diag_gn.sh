#!/bin/bash
# GPU box: GN-step timing (stamps of a continuing vs a stopping last level-0 pass, the lone-pair alignment) after
# the GPU tests.  usage: tools/diag_gn.sh <tag> [pytest args]
set -o pipefail
TAG=${1:-a}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/diag_$TAG; mkdir -p $O; cd $R
if [ "$1" != "--no-tests" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
export R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_stamps.so
ALIGN=1 timeout -k 10 120 python3 tools/stamps.py > $O/stamps_stop.txt 2>&1 || { tail $O/stamps_stop.txt; exit 1; }
ALIGN=1 R360_DIAG_EXTRA_ITERS=1 timeout -k 10 120 python3 tools/stamps.py > $O/stamps_cont.txt 2>&1 || { tail $O/stamps_cont.txt; exit 1; }
unset R360_LIB
timeout -k 10 120 python3 tools/lone_align.py 30 > $O/lone.txt 2>&1 || { tail $O/lone.txt; exit 1; }
grep -E "align last|eval at" $O/stamps_*.txt; tail -3 $O/lone.txt
