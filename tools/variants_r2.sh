# bench variants for the current build (via gpurun): tools/variants_r2.sh <outdir> "<name>:<args>" ...
set -o pipefail
OUT=gpurun_out/${1:-var}; shift
mkdir -p $OUT
for v in "$@"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-resident $a > $OUT/$n.json 2> $OUT/$n.err || { echo fail $n; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$n',round(d['value'],1),'P',d['config']['pipelines_per_gpu'],'L0',round(r['avg_launch_ms']*1e3,1),'us/launch',round(r['pairs_per_launch'],2),'pairs frac',round(r['frac'] or 0,3),{k:round(v,2) for k,v in d['pipeline_host_ms_per_pair'].items()})"
done
