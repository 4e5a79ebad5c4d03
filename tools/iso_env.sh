#!/bin/bash
# GPU box: isolated plane-half kernel times (tools/iso_trace.sh) under several environment settings.
# usage: tools/iso_env.sh "<ENV=..>" ...  ("-" = none); KERNELS = grep pattern of the rows to print
R=$GRAFT_REPO_ROOT; i=0
for e in "$@"; do
  i=$((i+1)); [ "$e" = "-" ] && e=""
  env $e bash $R/tools/iso_trace.sh env$i > /dev/null 2>&1 || { echo "[$e] failed"; exit 1; }
  echo "[$e] $(head -1 $R/gpurun_out/iso_env$i/plane_half.txt)"
  grep -E "${KERNELS:-k_}" $R/gpurun_out/iso_env$i/area.txt | head -${ROWS:-8}
done
