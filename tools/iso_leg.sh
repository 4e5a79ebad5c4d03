set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/iso; mkdir -p $O; cd $R
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-config5 --no-halves > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/b$i.json')); r=d['roofline']['isolated']
print('value %.1f lone median %.3f mean %.3f L0 %.2f us' % (d['value'], r['align_ms_per_pair'], r['align_ms_per_pair_mean'], r['avg_launch_ms']*1e3))"
done
