#!/bin/bash
# One development round trip on the GPU box (via gpurun, repo root): GPU tests, dense-alone VGA bench lines of
# the ICP pass forms given in PFS (in-kernel spans), their level-0 VALU / HBM counters, and the default bench.
# usage: PFS="4 5" tools/r3_iter.sh <tag> [skip-tests]
set -o pipefail
export R360_LIB=${R360_LIB:-${GRAFT_REPO_ROOT:-.}/rgbd360_amd/lib/librgbd360_hip_exp.so}   # knobs: experiment build (make -C rgbd360_amd/csrc exp)
TAG=${1:-it}; R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/it_$TAG; mkdir -p $OUT
DARGS="--workload dense --steps 2 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-isolated"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 420 python -u -m pytest $R/tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
cd /tmp && export TMPDIR=/tmp
for pf in ${PFS:-5}; do
  R360_ICP_PF=$pf timeout -k 10 200 python3 $R/bench.py $DARGS > $OUT/dense_pf$pf.json 2> $OUT/dense_pf$pf.err || { echo "dense pf$pf failed"; tail -5 $OUT/dense_pf$pf.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('$OUT/dense_pf$pf.json')); r=d['roofline']; print('PF $pf dense', round(d['value'],1), 'pairs/s; L0', round(r['avg_launch_ms']*1e3/r['pairs_per_launch'],2), 'us/pair-pass at', round(r['pairs_per_launch'],2), 'pairs/launch, frac', round(r['frac'],3))"
  R360_ICP_PF=$pf timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/prof_pf$pf/pmc1 -o p -- python3 $R/bench.py $DARGS > /dev/null 2> $OUT/pmc_pf$pf.err || { echo "pmc pf$pf failed"; exit 3; }
  R360_ICP_PF=$pf timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE SQ_WAVES -d $OUT/prof_pf$pf/pmc2 -o p -- python3 $R/bench.py $DARGS > /dev/null 2> $OUT/pmcb_pf$pf.err || { echo "pmcb pf$pf failed"; exit 3; }
  R360_ICP_PF=$pf timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE SQ_WAVES -d $OUT/prof_pf$pf/pmc3 -o p -- python3 $R/bench.py $DARGS > /dev/null 2> $OUT/pmcc_pf$pf.err || { echo "pmcc pf$pf failed"; exit 3; }
  python3 $R/tools/hires_summary.py $OUT/prof_pf$pf $OUT/dense_pf$pf.json > $OUT/pmc_pf$pf.json 2>&1
  python3 -c "import json; d=json.load(open('$OUT/pmc_pf$pf.json')); print('PF $pf per pair-pass: VALU', d['SQ_INSTS_VALU_per_pair_pass'], 'HBM', d.get('hbm_bytes_per_pair_pass'), 'alg', d.get('algorithmic_bytes_per_pair_pass'))"
  find $OUT -name "*.csv" -size +2M -delete
done
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python3 $R/bench.py $BENCH > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 4; }
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']; print('bench', round(d['value'],1), 'pairs/s, frac', round(r['frac'],3), 'iso', r['isolated']['frac'], 'c5', d.get('config5',{}).get('value'), d.get('config5',{}).get('roofline',{}).get('frac'))"
fi
