#!/bin/bash
# GPU box: frame-preparation kernel change: its parity tests, isolated kernel times of this tree and of build/ab_base,
# then the alternating default-bench A/B (tools/ab.sh).   usage: tools/r5_prep_ab.sh <tag>
set -o pipefail
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prep_$TAG; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_hires.py tests/test_gpu_pinhole.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/frame_iso.sh ${TAG}_new > $O/iso_new.txt 2>&1 || { tail $O/iso_new.txt; exit 2; }
GRAFT_REPO_ROOT=$R/build/ab_base bash tools/frame_iso.sh ${TAG}_base > $O/iso_base.txt 2>&1 || { tail $O/iso_base.txt; exit 3; }
paste <(head -25 $O/iso_new.txt) <(head -25 $O/iso_base.txt | cut -c62-)
bash tools/ab.sh $TAG build/ab_base
