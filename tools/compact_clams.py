"""Convert a CLAMS DiscreteDepthDistortionModel file (discrete_depth_distortion_model.cpp:259-280)
into the compact 'R360CLAMS1' table used by data/calib/Intrinsics: header + per-frustum per-bin
counts and multipliers (the only fields undistort() reads, :48-68).

usage: python tools/compact_clams.py <src_dir> <dst_dir>
"""
import struct
import sys

import numpy as np


def convert(src: str, dst: str) -> None:
    d = open(src, "rb").read()
    off = d.index(b"\n") + 1
    w, h, bw, bh = struct.unpack_from("<iiii", d, off); off += 16
    bd, = struct.unpack_from("<d", d, off); off += 8
    nx, ny = struct.unpack_from("<ii", d, off); off += 8
    counts, mult = [], []
    nb = 0
    for _ in range(nx * ny):
        _maxd, nb, _bdep = struct.unpack_from("<did", d, off); off += 20
        vecs = []
        for _q in range(4):
            _by, r, c = struct.unpack_from("<iii", d, off); off += 12
            vecs.append(np.frombuffer(d, np.float32, r * c, off)); off += 4 * r * c
        counts.append(vecs[0]); mult.append(vecs[3])
    assert off == len(d)
    with open(dst, "wb") as f:
        f.write(b"R360CLAMS1\n")
        f.write(struct.pack("<iiiiiiid", w, h, bw, bh, nx, ny, nb, bd))
        f.write(np.array(counts, np.float32).tobytes())
        f.write(np.array(mult, np.float32).tobytes())


if __name__ == "__main__":
    for k in range(1, 9):
        convert(f"{sys.argv[1]}/distortion_model{k}", f"{sys.argv[2]}/distortion_model{k}.r360")
