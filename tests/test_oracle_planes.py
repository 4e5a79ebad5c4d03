"""CPU checks of the oracle's plane half (A3-A9, A11-A13): hand-derived known answers for the
per-pixel stages, and an accuracy check of the full PbMap registration on a synthetic pair with a known
pose (accuracy, separate from GPU parity).  PCL/MRPT pieces are 'parity unpinned' (DESIGN.md §Oracle)."""
import numpy as np
import pytest

import rgbd360_amd as R
from oracle import oracle360 as O


def _plane_depth(rows, cols, n, d):
    """Depth image (metres) of the plane n.p + d = 0 seen by the reference pinhole (CloudRGBD_Ext.h:97-102)."""
    f = np.float32(525 * np.float32(cols / 640.0))
    ox, oy = cols // 2 - 0.5, rows // 2 - 0.5
    v, u = np.mgrid[0:rows, 0:cols].astype(np.float64)
    ray = np.stack([(u - ox) / f, (v - oy) / f, np.ones_like(u)], -1)
    z = -d / (ray @ np.asarray(n, np.float64))
    return z.astype(np.float32)


def test_cloud_downsample_upper_median_and_centre_rgb():
    rows, cols = 4, 4
    dm = np.array([[1.0, 2.0, 0.0, 0.0],
                   [3.0, 4.0, 0.0, 7.0],      # block (0,1): only z=7 (> maxDepth 5) -> copy centre point
                   [0.2, 1.5, 2.0, 2.0],      # 0.2 < minDepth: invalid
                   [1.0, 1.0, 2.0, 4.9]], np.float32)
    bgr = np.arange(rows * cols * 3, dtype=np.uint8).reshape(rows, cols, 3)
    xyz, rgb = O.cloud_downsample(dm, bgr)
    assert xyz.shape == (2, 2, 4)
    assert xyz[0, 0, 2] == np.float32(3.0)                 # sorted (1,2,3,4) -> element 2
    assert np.isfinite(xyz[0, 1, :3]).all() and xyz[0, 1, 2] == np.float32(7.0)   # centre (1,3) copied
    assert xyz[1, 0, 2] == np.float32(1.0)                 # (1.5, 1, 1) -> sorted (1, 1, 1.5)[1]
    assert xyz[1, 1, 2] == np.float32(2.0)
    c = bgr[1, 1]
    assert list(rgb[0, 0, :3]) == [c[2], c[1], c[0]]       # RGB from pixel (r+1, c+1), BGR swapped


def test_bilateral_constant_depth_is_fixed_point():
    xyz = np.zeros((40, 60, 4), np.float32)
    xyz[..., 2] = 2.5
    out = O.bilateral(xyz)
    assert np.allclose(out[..., 2], 2.5, atol=1e-6)
    xyz[5, 7, :3] = np.nan                                  # NaN z becomes max z first
    out = O.bilateral(xyz)
    assert np.isfinite(out[..., 2]).all() and np.isnan(out[5, 7, 0])


def test_normals_on_a_plane_and_borders():
    n = np.array([0.2, -0.1, -1.0]); n /= np.linalg.norm(n)
    dm = _plane_depth(240, 320, n, 2.0)
    xyz, _ = O.cloud_downsample(dm, np.zeros((240, 320, 3), np.uint8))
    nrm, dist = O.normals(xyz)
    assert np.isnan(nrm[:8, :, 0]).all() and np.isnan(nrm[:, -8:, 0]).all()
    inner = nrm[8:-8, 8:-8, :3]
    assert np.isfinite(inner).all()
    # flipped towards the viewpoint: n . (0 - p) >= 0
    assert np.allclose(np.abs(inner @ n), 1.0, atol=1e-4)
    assert (np.einsum("ijk,ijk->ij", inner, -xyz[8:-8, 8:-8, :3]) >= 0).all()


def test_segment_two_planes():
    rows, cols = 240, 320
    a = _plane_depth(rows, cols, [0.0, 0.3, -1.0], 2.0)
    b = _plane_depth(rows, cols, [0.5, 0.0, -1.0], 2.4)
    dm = a.copy()
    dm[:, cols // 2:] = b[:, cols // 2:]
    xyz, _ = O.cloud_downsample(dm, np.zeros((rows, cols, 3), np.uint8))
    xyz = O.bilateral(xyz)
    nrm, _ = O.normals(xyz)
    lc, lf, regs = O.segment(xyz, nrm)
    assert len(regs) == 2
    for r, nn in zip(sorted(regs, key=lambda r: r["centroid"][0]), ([0.0, 0.3, -1.0], [0.5, 0.0, -1.0])):
        nn = np.asarray(nn) / np.linalg.norm(nn)
        assert abs(abs(r["model"][:3] @ nn) - 1) < 1e-3
        assert r["curvature"] < 1e-3 and r["count"] > 1000
    # refinement only grows planar labels
    assert ((lf != lc) <= (lc >= 0)).all()


@pytest.fixture(scope="module")
def synth_pair():
    rt = O.read_extrinsics(R.EXTRINSICS_DIR)
    seed = 360 << 16
    A = R.synth_path_pose(seed, 0)
    rel = np.eye(4, dtype=np.float32)
    a = np.deg2rad(4.0)
    rel[1:3, 1:3] = [[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]]
    rel[:3, 3] = [0, 0.25, 0.15]
    maps = []
    for P in (A, A @ rel):
        b, d = R.synth_frame_rt(480, 640, rt, seed, P)
        maps.append(O.PbMap(d.astype(np.float32) * np.float32(0.001), b, rt))
    return maps, rel


def test_pbmap_planes_are_consistent(synth_pair):
    (m1, m2), _ = synth_pair
    for m in (m1, m2):
        P = m.planes()
        assert len(P) >= 8
        for p in P:
            assert abs(np.linalg.norm(p["normal"]) - 1) < 1e-5
            assert abs(p["d"] + p["normal"] @ p["center"]) < 1e-4
            assert p["area"] >= 0.12 and p["elongation"] <= 6
            assert np.allclose(p["hull"][0], p["hull"][-1])          # closed hull polygon


def test_register_pbmap_synthetic_accuracy(synth_pair):
    (m1, m2), rel = synth_pair
    r = O.register_pbmap(m1, m2, 25, O.PLANAR_3DoF)
    assert r["good"] == 1 and len(r["matches"]) >= 6
    assert np.rad2deg(O.rot_angle(r["pose"][:3, :3], rel[:3, :3])) < 0.3
    assert np.linalg.norm(r["pose"][:3, 3] - rel[:3, 3]) < 0.02
