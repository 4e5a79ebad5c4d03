"""Timeline of the last <k> pairs of a sequential-leg kernel trace (tools/seq_leg.py under rocprofv3
--kernel-trace --memory-copy-trace): every kernel / copy with its start offset from the pair's upload and its
duration, and per pair the spans of the dense preparation, the plane chain and the alignment.
usage: python tools/seq_chain.py <trace dir> [pairs to print, default 3]"""
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(k_\w+(?:<[^>]*>)?|__amd_\w+)", name)
    return m.group(1) if m else name[:50]


d = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ev = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                   r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?"),
                   "-", r.get("Stream_Id", "?")))
ev.sort()
# a pair starts at an upload-sized host-to-device copy (>= 1 MB: the 8 x 640 x 480 BGR + depth images) or, with
# device inputs, at the first k_undistort4 after an alignment; use k_undistort4 launches as pair boundaries
starts = [i for i, e in enumerate(ev) if e[2].startswith("k_undistort4")]
bounds = starts[-(K + 1):]
for a, b in zip(bounds[:-1], bounds[1:]):
    # back up to the copies right before the undistortion
    s = a
    while s > 0 and ev[s - 1][2].startswith("copy") and ev[a][0] - ev[s - 1][0] < 3000_000:
        s -= 1
    t0 = ev[s][0]
    print(f"---- pair (kernels {s}..{b - 1}), span to next undistort {(ev[b][0] - t0) / 1e3:.1f} us")
    for e in ev[s:b]:
        print(f"  {(e[0] - t0) / 1e3:8.1f} {(e[1] - t0) / 1e3:8.1f}  {(e[1] - e[0]) / 1e3:7.1f} us  q{e[3]:>3} s{e[4]:>3}  {e[2]}")
