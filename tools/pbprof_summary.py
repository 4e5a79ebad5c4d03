"""Mean of the [pbmap] phase lines an R360_PBMAP_PROFILE run prints (experiment builds):
python3 tools/pbprof_summary.py <stderr file>"""
import re
import sys

keys = ["sensors", "prefilter", "hull", "area+desc", "local merges", "groupPlanes", "mergePlanes", "models", "points",
        "voxels", "kept", "hull vertices", "planes"]
pat = re.compile(r"sensors ([\d.]+) us: prefilter ([\d.]+), hull ([\d.]+), area\+desc ([\d.]+), local merges ([\d.]+) \| "
                 r"groupPlanes ([\d.]+) us, mergePlanes ([\d.]+) us \| models (\d+), points (\d+) \(voxels (\d+)\) -> "
                 r"(\d+) kept -> (\d+) hull vertices, planes (\d+)")
rows = [list(map(float, m.groups())) for m in map(pat.search, open(sys.argv[1])) if m]
if not rows:
    sys.exit("no [pbmap] lines")
n = len(rows)
print(f"{n} frames; mean per frame:")
for k, v in zip(keys, zip(*rows)):
    print(f"  {k:14s} {sum(v) / n:10.1f}   (max {max(v):.0f})")
