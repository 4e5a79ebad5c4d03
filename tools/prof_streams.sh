#!/bin/bash
# GPU box: rocprofv3 kernel trace of the bench with S pipelines (round 2 recorded crashes of 16-pipeline traces).
# usage: tools/prof_streams.sh <streams> [tag]   -> gpurun_out/ps_<streams>[_tag]/{bench.json,trace.err,stats}
S=${1:-16}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ps_$S${2:+_$2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 -X faulthandler $R/bench.py --streams $S --steps 2 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-isolated > $O/bench.json 2> $O/trace.err
rc=$?
echo "rocprofv3 exit $rc"
tail -c 30000 $O/trace.err > $O/t && mv $O/t $O/trace.err
ls $O/trace/ 2>/dev/null | head; find $O/trace -name "*kernel_trace.csv" -exec rm -f {} \; 2>/dev/null
exit $rc
