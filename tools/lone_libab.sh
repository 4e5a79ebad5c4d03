# GPU box: tools/lone_align.py alternating two libraries, LONEAB="name1|name2" (rgbd360_amd/lib/librgbd360_<name>.so)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/lone_libab; mkdir -p $O; cd $R
IFS='|' read -ra LIBS <<< "${LONEAB:?LONEAB=name1|name2}"
for rep in 1 2 3; do
  for l in "${LIBS[@]}"; do
    echo "== $l rep $rep"
    R360_LIB=$R/rgbd360_amd/lib/librgbd360_$l.so timeout -k 10 120 python -u tools/lone_align.py 30 > $O/out.txt 2>&1 || { tail -20 $O/out.txt; exit 1; }
    tail -2 $O/out.txt | head -1
  done
done
