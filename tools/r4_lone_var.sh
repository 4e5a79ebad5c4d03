#!/bin/bash
# GPU box: the lone-pair alignment (tools/lone_align.py) under several library builds and knobs, one after another.
# usage: tools/r4_lone_var.sh <tag> "<lib-suffix>[:ENV=V]"...   (suffix "" = the product library)
set -o pipefail
TAG=${1:-v}; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lone_$TAG; mkdir -p $O; cd $R
i=0
for spec in "$@"; do
  suf=${spec%%:*}; env_=""; [ "$spec" != "$suf" ] && env_=${spec#*:}
  lib=$R/rgbd360_amd/lib/librgbd360_hip${suf:+_$suf}.so
  env R360_LIB=$lib $env_ timeout -k 10 120 python3 tools/lone_align.py 30 > $O/v$i.txt 2>&1 || { tail -5 $O/v$i.txt; exit 1; }
  echo "[$spec] $(tail -2 $O/v$i.txt | tr '\n' ' ')"
  i=$((i+1))
done
