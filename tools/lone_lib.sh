#!/bin/bash
# GPU box: tools/lone_align.py against several libraries (paths relative to the repo root)
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lonelib_$TAG; mkdir -p $O
cd $R
for v in "$@"; do
  IFS='|' read -r n lib e <<< "$v"
  env R360_LIB=$R/$lib $e timeout -k 10 120 python3 -u tools/lone_align.py 30 > $O/$n.txt 2>&1 || { echo "$n failed"; tail -5 $O/$n.txt; exit 1; }
  echo "== $n"; cat $O/$n.txt
done
