#!/bin/bash
# Kernel durations of the refinement sweeps on saved real-frame inputs (tmp_refine/*.npz, scratch), per variant
# given as "name:ENV=VAL ...".  usage (via gpurun): tools/refine_bench.sh <outdir> name:env...
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  for w in fire nofire; do
    timeout -k 10 120 env $envs rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${name}_$w -o t -- python3 $R/tmp_refine/fire2.py $w > /dev/null 2>&1 || exit 1
    echo "== $name $w" >> $OUT/summary.txt
    grep -h "refine" $OUT/${name}_$w/*kernel_stats.csv | cut -d, -f1-5 >> $OUT/summary.txt
    rm -f $OUT/${name}_$w/*trace.csv
  done
done
cat $OUT/summary.txt
