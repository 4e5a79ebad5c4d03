#!/bin/bash
# GPU box: one development step.  usage: tools/gpu_step.sh <tag> [stages...]
#   tests  every -m gpu test            smoke   __graft_entry__.smoke()
#   bench  the default bench line        quick   a short sequence-only bench line (no CPU / config-5 / halves legs)
#   pbprof PbMap assembly phase profile (experiment build, R360_PBMAP_PROFILE) over a short sequence run
#   c5     the config-5 leg alone (HiRes dense, 50 level-0 iterations)
# results in gpurun_out/<tag>/; every GPU step under its own time limit, the first failure ends the script
set -o pipefail
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
Q="--no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves"
for st in "$@"; do
  case $st in
    tests)
      R360_TEST_DRIFT_OUT=$O/drift timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 \
        || { tail -40 $O/gpu_tests.log; exit 1; }
      tail -2 $O/gpu_tests.log ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
      tail -2 $O/smoke.log ;;
    bench)
      timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
      python3 tools/bench_line.py $O/bench.json ;;
    quick)
      timeout -k 10 200 python -u bench.py $Q > $O/quick.json 2> $O/quick.err || { tail -20 $O/quick.err; exit 4; }
      python3 tools/bench_line.py $O/quick.json ;;
    pbprof)
      R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_exp.so R360_PBMAP_PROFILE=1 timeout -k 10 200 python -u bench.py $Q \
        --steps 2 --warmup 1 > $O/pbprof.json 2> $O/pbprof.err || { tail -20 $O/pbprof.err; exit 5; }
      grep -c '^\[pbmap\]' $O/pbprof.err; python3 tools/pbprof_summary.py $O/pbprof.err | tee $O/pbprof.txt ;;
    c5)
      timeout -k 10 300 python -u -c "
import json, sys; sys.argv=['bench.py']; import numpy as np, bench, rgbd360_amd as R
rt8 = np.stack([np.loadtxt(f'{R.EXTRINSICS_DIR}/Rt_0{k + 1}.txt', dtype=np.float32) for k in range(8)])
print(json.dumps(bench.config5_leg(0, rt8)))" > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 6; }
      python3 -c "import json; d=json.load(open('$O/c5.json')); r=d['roofline']; print('config5', round(d['value'],1), 'pairs/s frac', round(r['frac'],3), 'L0', round(r['avg_launch_ms']*1e3,1), 'us/launch', round(r['pairs_per_launch'],2), 'pairs/launch')" ;;
    envab)  # the default sequence line (quick legs) over environments of the experiment library, ENVAB="env1|env2|...", twice each
      IFS='|' read -ra ENVS <<< "${ENVAB:?ENVAB=env1|env2}"
      for rep in 1 2; do
        for i in "${!ENVS[@]}"; do
          env R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_exp.so ${ENVS[$i]} timeout -k 10 200 python -u bench.py $Q \
            > $O/ab_${i}_$rep.json 2> $O/ab_${i}_$rep.err || { tail -20 $O/ab_${i}_$rep.err; exit 10; }
          echo "== [${ENVS[$i]}] rep $rep"; python3 tools/bench_line.py $O/ab_${i}_$rep.json | head -2
        done
      done ;;
    trace)  # kernel trace of the default sequence line (quick legs): dense-stream gaps, GPU busy, per-kernel stats
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $O/trace -o trace -- python3 $R/bench.py $Q > $O/trace_bench.json 2> $O/trace.err ) \
        || { tail -20 $O/trace.err; exit 11; }
      T=$(ls $O/trace/*kernel_trace.csv | head -1)
      python3 tools/dense_gaps.py $T > $O/dense_gaps.txt && python3 tools/busy.py $T 1000 > $O/busy.txt \
        && cp $(ls $O/trace/*kernel_stats.csv | head -1) $O/kernel_stats.csv
      find $O/trace -name "*.csv" -delete
      head -8 $O/dense_gaps.txt; head -3 $O/busy.txt; python3 tools/bench_line.py $O/trace_bench.json | head -1 ;;
    seq)    # the sequential caller's leg alone, plane stage on the pipeline's stream (0) and on a plane queue (8)
      timeout -k 10 300 python -u -c "
import json, sys; sys.argv=['bench.py']; import numpy as np, bench, rgbd360_amd as R
rt8 = np.stack([np.loadtxt(f'{R.EXTRINSICS_DIR}/Rt_0{k + 1}.txt', dtype=np.float32) for k in range(8)])
BGR = np.zeros((40, 8, 480, 640, 3), np.uint8); DEP = np.zeros((40, 8, 480, 640), np.uint16)
for j in range(40): BGR[j], DEP[j] = R.synth_frame_rt(480, 640, rt8, bench.SEED, R.synth_path_pose(bench.SEED, j))
pin = R.HostPinned(BGR, DEP)
p = R.IcpParams.default(); p.n_pyr = 5; p.std_dev_photo = np.float32(3.0 / 255); p.fixed_iters_level0 = 20
out = {}
for rep in range(2):
    for pb in (0, 8):
        out[f'pb{pb}_{rep}'] = bench.sequential_leg(0, 480, 640, 0, lambda i: (BGR[i], DEP[i]), p, pairs=32, plane_batch=pb)
print(json.dumps(out))" > $O/seq.json 2> $O/seq.err || { tail -20 $O/seq.err; exit 12; }
      cat $O/seq.json ;;
    argab)  # the default sequence line (quick legs) over bench argument sets, ARGAB="args1|args2|...", twice each
      IFS='|' read -ra ARMS <<< "${ARGAB:?ARGAB=args1|args2}"
      for rep in 1 2; do
        for i in "${!ARMS[@]}"; do
          timeout -k 10 200 python -u bench.py $Q ${ARMS[$i]} > $O/arg_${i}_$rep.json 2> $O/arg_${i}_$rep.err \
            || { tail -20 $O/arg_${i}_$rep.err; exit 13; }
          echo "== [${ARMS[$i]}] rep $rep"; python3 tools/bench_line.py $O/arg_${i}_$rep.json | head -1
        done
      done ;;
    libab)  # the default sequence line (quick legs) alternating libraries, LIBAB="name1|name2" (rgbd360_amd/lib/librgbd360_<name>.so)
      IFS='|' read -ra LIBS <<< "${LIBAB:?LIBAB=name1|name2}"
      for rep in 1 2; do
        for l in "${LIBS[@]}"; do
          R360_LIB=$R/rgbd360_amd/lib/librgbd360_$l.so timeout -k 10 200 python -u bench.py $Q > $O/lib_${l}_$rep.json \
            2> $O/lib_${l}_$rep.err || { tail -20 $O/lib_${l}_$rep.err; exit 14; }
          echo "== $l rep $rep"; python3 tools/bench_line.py $O/lib_${l}_$rep.json | head -2
        done
      done ;;
    pfab)   # level-0 pass forms / occupancy: dense-alone VGA and config 5, per experiment library:PF (PFAB="exp:6 minb4:7")
      for spec in ${PFAB:-exp:6 minb4:7 minb4:6}; do
        lib=${spec%%:*}; pf=${spec##*:}; n=${lib}_pf$pf
        R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_$lib.so R360_ICP_PF=$pf timeout -k 10 200 python -u bench.py --workload dense \
          $Q > $O/dense_$n.json 2> $O/dense_$n.err || { tail -20 $O/dense_$n.err; exit 7; }
        echo "== $n dense"; python3 tools/bench_line.py $O/dense_$n.json | head -1
        R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_$lib.so R360_ICP_PF=$pf timeout -k 10 300 python -u -c "
import json, sys; sys.argv=['bench.py']; import numpy as np, bench, rgbd360_amd as R
rt8 = np.stack([np.loadtxt(f'{R.EXTRINSICS_DIR}/Rt_0{k + 1}.txt', dtype=np.float32) for k in range(8)])
print(json.dumps(bench.config5_leg(0, rt8)))" > $O/c5_$n.json 2> $O/c5_$n.err || { tail -20 $O/c5_$n.err; exit 8; }
        python3 -c "import json; d=json.load(open('$O/c5_$n.json')); r=d['roofline']; print('config5', round(d['value'],1), 'pairs/s frac', round(r['frac'],3), 'L0', round(r['avg_launch_ms']*1e3,1), 'us/launch', round(r['pairs_per_launch'],2), 'pairs/launch')"
      done ;;
    *) echo "unknown stage $st"; exit 9 ;;
  esac
done
