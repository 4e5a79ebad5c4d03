"""One-line summary of a bench.py JSON line: python3 tools/bench_line.py <bench.json>"""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"]
iso = r.get("isolated") or {}
c5 = d.get("config5") or {}
c5r = c5.get("roofline") or {}
hs = d.get("host_cores_split") or {}
print(f"value {d['value']:.1f} pairs/s  resident {d.get('value_hbm_resident_inputs') or 0:.1f}  "
      f"records_identical {d.get('records_identical')}  L0 frac {r['frac'] or 0:.3f} ({r['avg_launch_ms'] * 1e3:.1f} us x "
      f"{r['pairs_per_launch']:.2f} pairs)  traffic {r.get('traffic')}")
print(f"host_cores_busy {d.get('host_cores_busy')} split {hs}  asm/frame "
      f"{d['pipeline_host_ms_per_pair'].get('pbmap_assembly_per_frame', 0):.3f} ms")
if iso.get("align_ms_per_pair"):
    print(f"lone pair {iso['align_ms_per_pair']:.3f} ms  L0 {iso['avg_launch_ms'] * 1e3:.1f} us frac {iso.get('frac') or 0:.3f}")
if c5:
    print(f"config5 {c5['value']:.1f} pairs/s frac {c5r.get('frac') or 0:.3f}  ({c5r.get('avg_launch_ms', 0) * 1e3:.1f} us x "
          f"{c5r.get('pairs_per_launch', 0):.2f})")
for k in ("config2", "config3", "sequential_cpp", "config1", "cpu_baseline"):
    if d.get(k):
        v = d[k]
        print(k, {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()
                  if not isinstance(vv, (dict, list)) and kk not in ("workload", "sample", "note")})
print("matcher", d.get("pbmap_matcher"), "dense_queue", d.get("dense_queue"), "plane_queue", d.get("plane_queue"))
if d.get("coarse_levels"):
    print("coarse", {k: (v["launches"], round(v["avg_launch_us"], 1), v["pair_passes"], round(v["ms_per_step"], 1))
                     for k, v in d["coarse_levels"].items()}, "(launches, us, pair passes, ms/step)")
