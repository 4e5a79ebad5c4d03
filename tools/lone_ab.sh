set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lone_ab; mkdir -p $O; cd $R
for rep in 1 2; do
for e in "X=0" "R360_ICP_CAP=768" "R360_ICP_CAP=1024" "R360_ICP_CAP=1280" "R360_ICP_PF=6" "R360_ICP_PF=6 R360_ICP_CAP=1024"; do
  echo "== $e"
  env R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_exp.so $e timeout -k 10 120 python -u tools/lone_align.py 30 > $O/out.txt 2>&1 || { tail -20 $O/out.txt; exit 1; }
  tail -2 $O/out.txt
done
done
