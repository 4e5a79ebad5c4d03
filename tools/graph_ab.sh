#!/bin/bash
# GPU box: lone-pair alignFrames360 A/B — pass sequence replayed as a captured hipGraph (shipped default) vs one
# launch at a time (R360_NO_GRAPH=1) vs the polled-flag experiment build — plus per-level in-kernel stamps.
# usage: tools/graph_ab.sh <tag>     (results in gpurun_out/graph_<tag>/)
set -o pipefail
export R360_LIB=${R360_LIB:-${GRAFT_REPO_ROOT:-.}/rgbd360_amd/lib/librgbd360_hip_exp.so}   # knobs: experiment build (make -C rgbd360_amd/csrc exp)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/graph_${1:-ab}; mkdir -p $O; cd $R
L=$R/rgbd360_amd/lib
R360_LIB=$L/librgbd360_hip_stamps.so NB=512 timeout -k 10 120 python3 -u tools/stamps.py > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
head -5 $O/stamps.txt
for rep in 1 2; do
  timeout -k 10 120 python3 -u tools/lone_align.py 30 >> $O/lone.txt 2>&1 || { tail $O/lone.txt; exit 2; }
  R360_NO_GRAPH=1 timeout -k 10 120 python3 -u tools/lone_align.py 30 >> $O/lone.txt 2>&1 || { tail $O/lone.txt; exit 3; }
  R360_LIB=$L/librgbd360_hip_poll.so timeout -k 10 120 python3 -u tools/lone_align.py 30 >> $O/lone.txt 2>&1 || { tail $O/lone.txt; exit 4; }
done
cat $O/lone.txt
