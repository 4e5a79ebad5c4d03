set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/chain; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" $O/gpu_tests.log | tail -25
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 -u tools/lone_align.py 30 > $O/lone_prod.txt 2>&1 && cat $O/lone_prod.txt &&
bash tools/r5_lone.sh chain "nochain|R360_NO_CHAIN=1" "chain|" "nochain2|R360_NO_CHAIN=1" "chain2|"
