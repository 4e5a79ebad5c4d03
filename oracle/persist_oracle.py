"""Keyframe persistence ORACLE — TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker).

Independent numpy/pure-Python restatement of the reference's on-disk formats:

* Frame360 .bin archives (Frame360::serialize / loadFrame, include/Frame360.h:236-249, 332-345; cv::Mat
  records of OpenNI2_Grabber/third_party/cvSerialization/cvmat_serialization.h:21-55) including the
  timestamp digit matrix (OpenNI2_Grabber/FrameRGBD/SerializeFrameRGBD.h:47-89).  Pinned: the sample
  captures round-trip byte-identically (tests/test_oracle.py).
* Frame360::sphereCloud (buildSphereCloud, Frame360.h:467-519): per-sensor clouds transformed by
  pcl::transformPointCloud's float expression, concatenated, height = w, width = 8*h.
* PCD v0.7 for pcl::PointXYZRGBA (pcl::io::savePCDFile, Frame360.h:326; PCDReader, :190-192) — PCL
  1.7's pcd_io.cpp (PCDWriter::generateHeader / writeASCII / writeBinary / writeBinaryCompressed)
  and its vendored liblzf.  PCL is third-party and not vendored: **parity unpinned** (no .pcd
  fixture in the reference).
* The R360 PbMap file (savePlanes / loadPbMap, Frame360.h:195-210, 312-318).  MRPT's CSerializable
  layout is not restatable here (MRPT absent): **parity unpinned**; this reader parses the documented
  replacement format independently of the product's writer.
"""
from __future__ import annotations

import gzip
import struct

import numpy as np

# ---------------------------------------------------------------- .bin archive
PROLOGUE = struct.pack("<Q", 22) + b"serialization::archive" + bytes([9, 0, 4, 8, 4, 8, 1, 0, 0, 0, 0, 0, 0, 0, 0])


def timestamp_digits(number: int) -> bytes:
    """getMatrixNumberRepresentationOf_uint64_t (SerializeFrameRGBD.h:47-74), loop as written."""
    num_digits, aux = 0, number
    while aux > 0:
        num_digits += 1
        aux //= 10
    out = bytearray(num_digits)
    remainder = number
    for i in range(num_digits):
        if remainder == 0:
            break
        divisor = int(10.0 ** (num_digits - 1 - i))  # pow(10, .) in double, converted to uint64
        quotient = remainder // divisor
        out[i] = quotient & 0xFF
        remainder = remainder - divisor * quotient
    return bytes(out)


def timestamp_value(digits: bytes) -> int:
    """get_uint64_t_ofMatrixRepresentation (SerializeFrameRGBD.h:77-89)."""
    number, p10 = 0, 1
    for d in reversed(digits):
        number = (number + p10 * d) & 0xFFFFFFFFFFFFFFFF
        p10 = (p10 * 10) & 0xFFFFFFFFFFFFFFFF
    return number


def _mat(cols: int, rows: int, esz: int, etype: int, data: bytes = b"") -> bytes:
    return struct.pack("<iiQQ", cols, rows, esz, etype) + data


def bin_bytes(bgr: np.ndarray, dep: np.ndarray, timestamp: int = 0) -> bytes:
    """Frame360::serialize: 8 x {CV_8UC3 (type 16), CV_16UC1 (type 2)} + timestamp mat (CV_8U, type 0).
    A zero timestamp is the empty mat the sample captures hold."""
    _, rows, cols = dep.shape
    parts = [PROLOGUE]
    for s in range(8):
        parts.append(_mat(cols, rows, 3, 16, np.ascontiguousarray(bgr[s], np.uint8).tobytes()))
        parts.append(_mat(cols, rows, 2, 2, np.ascontiguousarray(dep[s], "<u2").tobytes()))
    dig = timestamp_digits(timestamp)
    parts.append(_mat(len(dig), 1, 1, 0, dig) if dig else _mat(0, 0, 0, 0))
    return b"".join(parts)


def parse_bin(b: bytes):
    """-> (bgr [8,r,c,3], depth [8,r,c], timestamp)."""
    assert b[:len(PROLOGUE) - 15] == PROLOGUE[:-15]
    off = len(PROLOGUE)
    bgr, dep = [], []
    for s in range(8):
        for m in range(2):
            c, r, esz, et = struct.unpack_from("<iiQQ", b, off)
            off += 24
            n = c * r * esz
            a = np.frombuffer(b, np.uint8, n, off)
            off += n
            if m == 0:
                assert (esz, et) == (3, 16)
                bgr.append(a.reshape(r, c, 3))
            else:
                assert (esz, et) == (2, 2)
                dep.append(a.view("<u2").reshape(r, c))
    ts = 0
    if off + 24 <= len(b):
        c, r, esz, et = struct.unpack_from("<iiQQ", b, off)
        off += 24
        if c > 0 and r > 0 and esz == 1:
            ts = timestamp_value(b[off:off + c * r])
    return np.stack(bgr), np.stack(dep), ts


# ---------------------------------------------------------------- sphereCloud
def sphere_cloud(xyz4: np.ndarray, rgb4: np.ndarray, rt: np.ndarray):
    """buildSphereCloud: xyz4 [8,h,w,4] sensor-frame clouds, rgb4 [8,h,w,4] = (r,g,b,a), rt [8,4,4] row-major.
    transformPointCloud (PCL 1.7 transforms.hpp): out_k = m(k,0)*x + m(k,1)*y + m(k,2)*z + m(k,3) in
    float, left to right; non-finite points are left as they were.  -> (xyz [n,3], rgba [n], width, height)."""
    S, h, w, _ = xyz4.shape
    out = np.empty((S, h * w, 3), np.float32)
    for s in range(S):
        p = xyz4[s].reshape(-1, 4)[:, :3].astype(np.float32)
        m = rt[s].astype(np.float32)
        fin = np.isfinite(p).all(axis=1)
        o = p.copy()
        for k in range(3):
            a = m[k, 0] * p[:, 0]
            a = a + m[k, 1] * p[:, 1]
            a = a + m[k, 2] * p[:, 2]
            a = a + m[k, 3]
            o[fin, k] = a[fin]
        out[s] = o
    c = rgb4.reshape(-1, 4).astype(np.uint32)
    rgba = c[:, 2] | (c[:, 1] << 8) | (c[:, 0] << 16) | (c[:, 3] << 24)
    return out.reshape(-1, 3), rgba.astype(np.uint32), S * h, w


# ---------------------------------------------------------------- PCD
def pcd_header(width: int, height: int, data: str) -> bytes:
    """PCDWriter::generateHeader for PointXYZRGBA + the DATA line its writers append."""
    return ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z rgba\nSIZE 4 4 4 4\n"
            "TYPE F F F U\nCOUNT 1 1 1 1\n"
            f"WIDTH {width}\nHEIGHT {height}\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {width * height}\nDATA {data}\n"
            ).encode()


def _g8(v: np.float32) -> str:
    # std::ostream with precision(8) and the default floatfield is printf's %.8g; NaN is "nan"
    return "nan" if np.isnan(v) else "%.8g" % float(v)


def pcd_bytes(xyz: np.ndarray, rgba: np.ndarray, width: int, height: int, mode: int = 0) -> bytes:
    xyz = np.asarray(xyz, np.float32).reshape(-1, 3)
    rgba = np.asarray(rgba, np.uint32).reshape(-1)
    if mode == 0:  # writeASCII: "v v v c" per point, trailing space trimmed
        lines = [f"{_g8(p[0])} {_g8(p[1])} {_g8(p[2])} {int(c)}\n" for p, c in zip(xyz, rgba)]
        return pcd_header(width, height, "ascii") + "".join(lines).encode()
    rec = np.zeros(len(xyz), dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("rgba", "<u4")])
    rec["x"], rec["y"], rec["z"], rec["rgba"] = xyz[:, 0], xyz[:, 1], xyz[:, 2], rgba
    if mode == 1:  # writeBinary: fields packed per point
        return pcd_header(width, height, "binary") + rec.tobytes()
    # writeBinaryCompressed: each field for all points, then LZF, preceded by the two sizes
    soa = b"".join(rec[f].tobytes() for f in ("x", "y", "z", "rgba"))
    z = lzf_compress(soa)
    return pcd_header(width, height, "binary_compressed") + struct.pack("<II", len(z), len(soa)) + z


def pcd_parse(b: bytes):
    """-> (xyz [n,3] f32, rgba [n] u32, width, height) for the x y z rgba layouts written above."""
    off, hdr = 0, {}
    while True:
        e = b.index(b"\n", off)
        line = b[off:e].decode().strip()
        off = e + 1
        if not line or line.startswith("#"):
            continue
        k, _, v = line.partition(" ")
        hdr[k] = v
        if k == "DATA":
            break
    assert hdr["FIELDS"].split() == ["x", "y", "z", "rgba"], hdr["FIELDS"]
    w, h = int(hdr["WIDTH"]), int(hdr["HEIGHT"])
    n = int(hdr.get("POINTS", w * h))
    if hdr["DATA"] == "ascii":
        rows = b[off:].decode().split("\n")[:n]
        xyz = np.array([[np.float32(t) for t in r.split()[:3]] for r in rows], np.float32).reshape(n, 3)
        rgba = np.array([int(r.split()[3]) for r in rows], np.uint32)
        return xyz, rgba, w, h
    if hdr["DATA"] == "binary":
        a = np.frombuffer(b, "<u4", 4 * n, off).reshape(n, 4)
    else:
        zs, us = struct.unpack_from("<II", b, off)
        soa = lzf_decompress(b[off + 8:off + 8 + zs], us)
        a = np.frombuffer(soa, "<u4").reshape(4, n).T
    return a[:, :3].copy().view(np.float32), a[:, 3].copy(), w, h


# ---------------------------------------------------------------- LZF (liblzf 3.x stream format)
def lzf_decompress(z: bytes, out_len: int) -> bytes:
    out = bytearray()
    i = 0
    while i < len(z):
        c = z[i]
        i += 1
        if c < 32:
            out += z[i:i + c + 1]
            i += c + 1
        else:
            ln = c >> 5
            if ln == 7:
                ln += z[i]
                i += 1
            ref = len(out) - ((c & 31) << 8) - z[i] - 1
            i += 1
            assert ref >= 0, "LZF back-reference before start"
            for k in range(ln + 2):
                out.append(out[ref + k])
    assert len(out) == out_len, (len(out), out_len)
    return bytes(out)


def lzf_compress(data: bytes) -> bytes:
    """A valid LZF stream: longest match over a 3-byte hash chain (depth 8), literal runs <= 32."""
    out = bytearray()
    chains: dict[bytes, list[int]] = {}
    lit = bytearray()
    n, i = len(data), 0

    def flush():
        for s in range(0, len(lit), 32):
            run = lit[s:s + 32]
            out.append(len(run) - 1)
            out.extend(run)
        lit.clear()

    while i < n:
        best_len, best_ref = 0, -1
        if i + 2 < n:
            key = data[i:i + 3]
            for ref in reversed(chains.get(key, [])[-8:]):
                if i - ref > 8192:
                    break
                ln = 3
                mx = min(264, n - i)
                while ln < mx and data[ref + ln] == data[i + ln]:
                    ln += 1
                if ln > best_len:
                    best_len, best_ref = ln, ref
            chains.setdefault(key, []).append(i)
        if best_len >= 3:
            flush()
            off, ln = i - best_ref - 1, best_len - 2
            if ln < 7:
                out.append((off >> 8) + (ln << 5))
            else:
                out.append((off >> 8) + (7 << 5))
                out.append(ln - 7)
            out.append(off & 255)
            for k in range(i + 1, min(i + best_len, n - 2)):
                chains.setdefault(data[k:k + 3], []).append(k)
            i += best_len
        else:
            lit.append(data[i])
            i += 1
    flush()
    return bytes(out)


# ---------------------------------------------------------------- R360 PbMap file
def pbmap_parse(path: str) -> list[dict]:
    with gzip.open(path, "rb") as f:
        b = f.read()
    assert b[:8] == b"R360PBM1", b[:8]
    version, n = struct.unpack_from("<II", b, 8)
    assert version == 1
    off, planes = 16, []
    for _ in range(n):
        pid, sensor = struct.unpack_from("<ii", b, off)
        off += 8
        fl = struct.unpack_from("<17f", b, off)
        off += 68
        cnt = struct.unpack_from("<q", b, off)[0]
        s1 = struct.unpack_from("<3q", b, off + 8)
        off += 32
        s2 = [int.from_bytes(b[off + 16 * k:off + 16 * k + 16], "little", signed=True) for k in range(6)]
        off += 96
        c = struct.unpack_from("<4q", b, off)
        off += 32
        (ll,) = struct.unpack_from("<I", b, off)
        label = b[off + 4:off + 4 + ll].decode()
        off += 4 + ll
        (nh,) = struct.unpack_from("<I", b, off)
        hull = np.frombuffer(b, "<f4", 3 * nh, off + 4).reshape(nh, 3)
        off += 4 + 12 * nh
        planes.append(dict(id=pid, sensor=sensor, normal=np.array(fl[0:3], np.float32),
                           center=np.array(fl[3:6], np.float32), ppal=np.array(fl[6:9], np.float32),
                           d=np.float32(fl[9]), area=np.float32(fl[10]), elongation=np.float32(fl[11]),
                           curvature=np.float32(fl[12]), nrgb=np.array(fl[13:16], np.float32),
                           intensity=np.float32(fl[16]), n_inliers=cnt, s1=s1, s2=s2, c=c, label=label,
                           hull=hull.copy()))
    assert off == len(b), "trailing bytes in PbMap file"
    return planes
