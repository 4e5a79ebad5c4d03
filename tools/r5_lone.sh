#!/bin/bash
# GPU box: lone-pair variants (tools/lone_align.py) by environment, then the GPU suite and default bench lines.
# usage: tools/r5_lone.sh <tag> "<name>|<env>" ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lone_$TAG; mkdir -p $O
cd $R
for v in "$@"; do
  IFS='|' read -r n e <<< "$v"
  env R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_exp.so $e timeout -k 10 120 python3 -u tools/lone_align.py 30 > $O/$n.txt 2>&1 || { echo "$n failed"; tail -5 $O/$n.txt; exit 1; }
  echo "== $n"; cat $O/$n.txt
done
