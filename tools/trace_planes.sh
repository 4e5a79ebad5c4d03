#!/bin/bash
# GPU box: kernel trace of the planes-alone workload (config 2: the plane stage of the sequence, batched on the plane
# queue), with per-kernel totals (tools/busy.py) and the bench line.
TAG=$1; shift; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/trp_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --workload planes --steps 3 --warmup 1 --no-cpu-baseline --no-resident --no-config5 --no-isolated --no-halves "$@" > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/busy.py $f 600 45 > $O/busy.txt && python3 $R/tools/kernel_area.py $f > $O/area.txt
python3 -c "import json; d=json.load(open('$O/bench.json')); print('planes', round(d['value'],1), d.get('plane_queue'))"
head -48 $O/busy.txt
rm -f $f
