set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/st_r5; mkdir -p $O; cd $R
R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_stamps.so NB=512 timeout -k 10 120 python3 tools/stamps.py > $O/eval.txt 2>&1 || { tail $O/eval.txt; exit 2; }
R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_stamps.so NB=512 ALIGN=1 timeout -k 10 120 python3 tools/stamps.py > $O/align.txt 2>&1 || { tail $O/align.txt; exit 2; }
cat $O/eval.txt; grep -E "align last|eval at" $O/align.txt
