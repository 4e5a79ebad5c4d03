set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/st_e; mkdir -p $O; cd $R
R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_stamps.so ALIGN=1 R360_DIAG_EXTRA_ITERS=1 timeout -k 10 120 python3 tools/stamps.py > $O/stamps_cont.txt 2>&1 || { tail $O/stamps_cont.txt; exit 2; }
grep -E "align last|eval at" $O/stamps_cont.txt
