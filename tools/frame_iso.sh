#!/bin/bash
# GPU box: isolated frame-build kernel durations (tools/frame_iso.py under rocprofv3 --kernel-trace --stats)
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/iso_$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/tools/frame_iso.py 40 > $O/out.txt 2>&1 || { tail -20 $O/out.txt; exit 1; }
cat $O/out.txt | tail -2
S=$(find $O/trace -name "*kernel_stats.csv" | head -1); cp $S $O/kernel_stats.csv
python3 - $O/kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:45]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.2f} us')
PY
find $O/trace -name "*.csv" -size +2M -delete
