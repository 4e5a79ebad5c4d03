#!/bin/bash
# GPU box: rocprofv3 kernel trace of the lone-pair alignFrames360 (tools/lone_align.py), per-launch durations of the
# level-0 pass against the in-kernel spans the library reports.  usage: tools/lone_trace.sh <tag>
set -o pipefail
export R360_LIB=${R360_LIB:-${GRAFT_REPO_ROOT:-.}/rgbd360_amd/lib/librgbd360_hip_exp.so}   # knobs: experiment build (make -C rgbd360_amd/csrc exp)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lone_trace_${1:-a}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for g in 0 1; do
  R360_NO_GRAPH=$g timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g$g -o t -- python3 $R/tools/lone_align.py 30 > $O/g$g.out 2> $O/g$g.err || { tail $O/g$g.err; exit 1; }
  cat $O/g$g.out
  S=$(ls $O/g$g/*kernel_stats.csv | head -1); grep -E "k_icp_pass" $S | cut -c1-200
done
