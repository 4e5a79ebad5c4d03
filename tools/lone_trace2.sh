#!/bin/bash
# GPU box: kernel + memory-copy trace of tools/lone_align.py (product library), for the per-alignment timeline.
# usage: tools/lone_trace2.sh <tag>   (results in gpurun_out/lt2_<tag>/)
set -o pipefail
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lt2_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o tr -- python3 $R/tools/lone_align.py 10 > $O/out.txt 2>&1 || { tail -20 $O/out.txt; exit 1; }
cd $R
python3 tools/lone_timeline.py $O/tr > $O/timeline.txt 2>&1; cat $O/timeline.txt
find $O -name "*.csv" -size +2M -delete
