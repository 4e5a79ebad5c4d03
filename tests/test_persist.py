"""Keyframe persistence on CPU (no GPU): the host-only codecs of librgbd360_hip.so (PCD writer /
reader, LZF) against the independent restatement in oracle/persist_oracle.py, and the .bin timestamp
matrix against the sample captures.  Frame-level save/load (which downloads from HBM) is covered by
tests/test_gpu_persist.py."""
import os

import numpy as np
import pytest

import rgbd360_amd as R
from oracle import persist_oracle as PO


def _cloud(n, seed=0, nan_frac=0.2):
    rng = np.random.default_rng(seed)
    xyz = (rng.standard_normal((n, 3)) * rng.choice([1e-6, 0.01, 1.0, 7.5, 1e4], (n, 1))).astype(np.float32)
    xyz[rng.random(n) < nan_frac] = np.nan
    rgba = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    # a run of repeated points so LZF has back-references to take
    xyz[n // 3:n // 3 + 64] = xyz[0]
    rgba[n // 3:n // 3 + 64] = rgba[0]
    return xyz, rgba


def _same(a, b):
    return np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


# ------------------------------------------------------------------ .bin timestamp matrix
@pytest.mark.parametrize("ts", [0, 7, 10, 1234567890123, 1418400000000000000, 2**64 - 1])
def test_timestamp_digit_matrix(ts):
    d = PO.timestamp_digits(ts)
    assert d == (bytes(int(c) for c in str(ts)) if ts else b"")
    assert PO.timestamp_value(d) == ts


def test_bin_archive_bytes_with_timestamp(data_dir):
    path = os.path.join(data_dir, "samples", "sphere_images_1.bin")
    raw = open(path, "rb").read()
    bgr, dep, ts = PO.parse_bin(raw)
    assert ts == 0 and bgr.shape == (8, 240, 320, 3)
    assert PO.bin_bytes(bgr, dep, 0) == raw          # zero timestamp = the samples' empty mat
    b = PO.bin_bytes(bgr, dep, 1418400123456)
    assert b[:len(raw) - 24] == raw[:-24]
    assert PO.parse_bin(b)[2] == 1418400123456


# ------------------------------------------------------------------ PCD codec
def test_pcd_ascii_bytes_match_pcl_writer(tmp_path):
    xyz, rgba = _cloud(3000, seed=1)
    xyz[5] = [np.float32(1.17549435e-38), np.float32(-3.4028235e38), np.float32(1.0 / 3.0)]
    p = str(tmp_path / "a.pcd")
    R.pcd_write(p, xyz, rgba, 60, 50, R.PCD_ASCII)
    assert open(p, "rb").read() == PO.pcd_bytes(xyz, rgba, 60, 50, 0)


@pytest.mark.parametrize("mode", [R.PCD_ASCII, R.PCD_BINARY, R.PCD_BINARY_COMPRESSED])
def test_pcd_roundtrip(tmp_path, mode):
    xyz, rgba = _cloud(4096, seed=2 + mode)
    p = str(tmp_path / "c.pcd")
    R.pcd_write(p, xyz, rgba, 64, 64, mode)
    x2, c2, w, h = R.pcd_read(p)
    assert (w, h) == (64, 64)
    assert np.array_equal(c2, rgba)
    if mode == R.PCD_ASCII:  # %.8g is not always round-trip exact for float32 (9 digits are)
        fin = np.isfinite(xyz)
        assert np.array_equal(np.isnan(x2), np.isnan(xyz))
        assert np.allclose(x2[fin], xyz[fin], rtol=1e-7, atol=0)
        assert _same(x2, PO.pcd_parse(open(p, "rb").read())[0])
    else:
        assert _same(x2, xyz)
        ox, oc, ow, oh = PO.pcd_parse(open(p, "rb").read())
        assert _same(ox, xyz) and np.array_equal(oc, rgba) and (ow, oh) == (64, 64)
    if mode == R.PCD_BINARY:
        assert open(p, "rb").read() == PO.pcd_bytes(xyz, rgba, 64, 64, 1)


def test_pcd_reads_other_lzf_streams(tmp_path):
    """The oracle's LZF (hash chains, longest match) makes a different valid stream; the product's
    decoder must read it, and the product's stream must decode with the oracle's decoder."""
    xyz, rgba = _cloud(2500, seed=7, nan_frac=0.5)
    p = str(tmp_path / "o.pcd")
    b = PO.pcd_bytes(xyz, rgba, 2500, 1, 2)
    open(p, "wb").write(b)
    x2, c2, w, h = R.pcd_read(p)
    assert _same(x2, xyz) and np.array_equal(c2, rgba) and (w, h) == (2500, 1)
    q = str(tmp_path / "p.pcd")
    R.pcd_write(q, xyz, rgba, 2500, 1, R.PCD_BINARY_COMPRESSED)
    qb = open(q, "rb").read()
    assert len(qb) < 16 * 2500  # the NaN / repeated runs compress
    assert _same(PO.pcd_parse(qb)[0], xyz)


def test_pcd_reader_field_layouts(tmp_path):
    """PCL clouds of other point types: PointXYZRGB (rgb packed in a float), extra fields, normals."""
    n = 40
    xyz, rgba = _cloud(n, seed=9, nan_frac=0.0)
    rec = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("rgb", "<u4"), ("normal_x", "<f4"),
                             ("curv", "<f8")])
    rec["x"], rec["y"], rec["z"], rec["rgb"] = xyz[:, 0], xyz[:, 1], xyz[:, 2], rgba
    hdr = (f"# .PCD v0.7\nVERSION 0.7\nFIELDS x y z rgb normal_x curv\nSIZE 4 4 4 4 4 8\nTYPE F F F F F F\n"
           f"COUNT 1 1 1 1 1 1\nWIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\nDATA binary\n").encode()
    p = str(tmp_path / "rgb.pcd")
    open(p, "wb").write(hdr + rec.tobytes())
    x2, c2, _, _ = R.pcd_read(p)
    assert _same(x2, xyz) and np.array_equal(c2, rgba)
    # ascii, no colour field, a 3-count field, CRLF line ends
    lines = "".join(f"{a:.9g} {b:.9g} {c:.9g} 1 2 3\r\n" for a, b, c in xyz)
    hdr = (f"VERSION .7\r\nFIELDS x y z v\r\nSIZE 4 4 4 4\r\nTYPE F F F I\r\nCOUNT 1 1 1 3\r\nWIDTH {n}\r\n"
           f"HEIGHT 1\r\nDATA ascii\r\n")
    open(p, "w", newline="").write(hdr + lines)
    x2, c2, _, _ = R.pcd_read(p)
    assert _same(x2, xyz) and not c2.any()


def test_pcd_empty_and_errors(tmp_path):
    p = str(tmp_path / "e.pcd")
    R.pcd_write(p, np.zeros((0, 3), np.float32), None, 0, 0, R.PCD_BINARY_COMPRESSED)
    x, c, w, h = R.pcd_read(p)
    assert x.shape == (0, 3) and (w, h) == (0, 0)
    xyz, rgba = _cloud(100, seed=3)
    R.pcd_write(p, xyz, rgba, 100, 1, R.PCD_BINARY)
    b = open(p, "rb").read()
    open(p, "wb").write(b[:-7])
    with pytest.raises(RuntimeError, match="truncated"):
        R.pcd_read(p)
    # a compressed block whose first token is a back-reference before the start of the output
    hdr = PO.pcd_header(100, 1, "binary_compressed")
    open(p, "wb").write(hdr + np.array([3, 1600], "<u4").tobytes() + bytes([0xE0, 0x05, 0x00]))
    with pytest.raises(RuntimeError, match="LZF"):
        R.pcd_read(p)
    open(p, "wb").write(hdr + np.array([3, 1599], "<u4").tobytes() + bytes([0x01, 0x05, 0x00]))
    with pytest.raises(RuntimeError, match="bad compressed block"):
        R.pcd_read(p)
    with pytest.raises(RuntimeError, match="cannot open"):
        R.pcd_read(str(tmp_path / "missing.pcd"))
