# GPU box: full-pipeline bench.py under ICP grid-cap variants (R360_ICP_CAP), results in gpurun_out/pexp/
set -e
export R360_LIB=${R360_LIB:-${GRAFT_REPO_ROOT:-.}/rgbd360_amd/lib/librgbd360_hip_exp.so}   # knobs: experiment build (make -C rgbd360_amd/csrc exp)
mkdir -p gpurun_out/pexp
B="timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20"
for rep in 1 2; do
  for cap in ${CAPS:-0 128 256}; do
    if [ $cap = 0 ]; then $B > gpurun_out/pexp/c${cap}_$rep.json 2> gpurun_out/pexp/c${cap}_$rep.err
    else R360_ICP_CAP=$cap $B > gpurun_out/pexp/c${cap}_$rep.json 2> gpurun_out/pexp/c${cap}_$rep.err; fi
  done
done
