set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pfab; mkdir -p $O; cd $R
for pf in 5 6; do
R360_LIB=$R/rgbd360_amd/lib/librgbd360_hip_exp.so R360_ICP_PF=$pf timeout -k 10 120 python3 -u tools/pf_ab.py > $O/pf$pf.txt 2>&1 || { tail $O/pf$pf.txt; exit 2; }
done
diff $O/pf5.txt $O/pf6.txt > $O/diff.txt; cat $O/diff.txt | head -60; exit 0
