set -o pipefail
mkdir -p gpurun_out/var3
for v in "planes:--workload planes" "dense:--workload dense" "s8:--streams 8" "q0:--queue 0"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-resident $a > gpurun_out/var3/$n.json 2> gpurun_out/var3/$n.err || { echo fail $n; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/var3/$n.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$n',round(d['value'],1),r['avg_launch_ms'],r['pairs_per_launch'],r['frac'],d['pipeline_host_ms_per_pair'])"
done
