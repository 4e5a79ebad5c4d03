set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/bl; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/env_ab.sh bl "fused|R360_BIL_FUSED=1" "axes|R360_BIL_FUSED=0"
