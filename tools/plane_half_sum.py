"""Per-frame plane-half kernel time from a tools/busy.py summary of an isolated (--streams 1) trace:
sums every kernel except the dense half's (ICP passes, stitch, pyramid, gradient, source compaction,
undistort shared by both halves is counted as plane half input).  usage: python tools/plane_half_sum.py busy.txt"""
import re
import sys

DENSE = ("k_icp_pass", "k_stitch", "k_pyramid", "k_gradient", "k_src_", "k_sensor_level0", "__amd_rocclr",
         "k_occ", "k_match_tables")
tot, frames, rows = 0.0, None, []
for line in open(sys.argv[1]):
    m = re.match(r"\s+([\d.]+) ms\s+(\d+) x\s+([\d.]+) us\s+(\S+)", line)
    if not m:
        continue
    ms, n, us, name = float(m.group(1)), int(m.group(2)), float(m.group(3)), m.group(4)
    if name == "k_cloud":
        frames = n
    if any(name.startswith(d) for d in DENSE):
        continue
    rows.append((ms, name))
    tot += ms
frames = frames or 1
print(f"plane half: {tot / frames * 1e3:.0f} us per frame over {frames} frames")
for ms, name in sorted(rows, reverse=True):
    print(f"  {ms / frames * 1e3:8.1f} us  {name}")
