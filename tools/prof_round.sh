set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/profile.sh ${TAG:-r1} || exit 1
mkdir -p $R/gpurun_out/summ_${TAG:-r1}
python3 $R/tools/profile_summary.py $R/gpurun_out/prof_${TAG:-r1} $R/gpurun_out/summ_${TAG:-r1} > $R/gpurun_out/summ_${TAG:-r1}/summary.txt 2>&1 || { rm -rf $R/gpurun_out/prof_${TAG:-r1}; exit 2; }
python3 $R/tools/busy.py $(ls $R/gpurun_out/prof_${TAG:-r1}/trace/*kernel_trace.csv | head -1) 250 > $R/gpurun_out/summ_${TAG:-r1}/busy.txt 2>&1
cp $R/gpurun_out/prof_${TAG:-r1}/trace_bench.json $R/gpurun_out/summ_${TAG:-r1}/ 2>/dev/null
rm -rf $R/gpurun_out/prof_${TAG:-r1}
cd $R && timeout -k 10 300 python3 bench.py > gpurun_out/summ_${TAG:-r1}/bench.json 2> gpurun_out/summ_${TAG:-r1}/bench.err || exit 3
echo all-done
