#!/bin/bash
# GPU box: the -m gpu suite, tools/lone_align.py twice (product library) and the bench's isolated leg twice.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/wait; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for i in 1 2; do timeout -k 10 120 python3 -u tools/lone_align.py 30 > $O/lone$i.txt 2>&1 || exit 2; head -1 $O/lone$i.txt | cut -c1-90; done
bash tools/iso_leg.sh
