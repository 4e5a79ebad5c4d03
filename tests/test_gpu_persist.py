"""GPU tests of keyframe persistence through the C-ABI:

* Frame360::serialize writes the raw images it loaded back byte-identically to the sample capture,
  and the timestamp digit matrix of oracle/persist_oracle.py;
* Frame360::sphereCloud equals the oracle's buildSphereCloud (transformPointCloud in float, bitwise)
  of the per-sensor clouds the plane stage holds in HBM;
* save(path, i) writes the PCD bytes the oracle's PCL-writer restatement produces and a PbMap file
  the oracle's independent reader parses to the frame's planes; load_PbMap_Cloud into a fresh frame
  restores planes, labels and cloud exactly, and RegisterPbMap on loaded maps equals RegisterPbMap on
  the built ones bit for bit.
MRPT's own .pbmap byte layout is not restated (parity unpinned)."""
import gzip
import os

import numpy as np
import pytest

import rgbd360_amd as R
from oracle import oracle360 as O
from oracle import persist_oracle as PO

pytestmark = pytest.mark.gpu

SAMPLES = ("sphere_images_1.bin", "sphere_images_10.bin")


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.fixture(scope="module")
def ctx():
    return R.Context(0)


@pytest.fixture(scope="module")
def rig(ctx):
    cal = R.Calib360(ctx, 240, 320)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    cal.loadIntrinsicCalibration(R.INTRINSICS_DIR)
    frames = []
    for name in SAMPLES:
        f = R.Frame360(cal)
        f.loadFrame(os.path.join(R.SAMPLES_DIR, name))
        f.getPlanes()
        frames.append(f)
    return dict(cal=cal, frames=frames, rt=O.read_extrinsics(R.EXTRINSICS_DIR))


def test_serialize_roundtrip_bytes_and_timestamp(rig, tmp_path):
    cal = rig["cal"]
    src = os.path.join(R.SAMPLES_DIR, SAMPLES[0])
    raw = open(src, "rb").read()
    f = rig["frames"][0]
    assert f.timeStamp == 0
    out = str(tmp_path / "f.bin")
    f.serialize(out)
    assert open(out, "rb").read() == raw
    ts = 1418400123456789
    f.setTimeStamp(ts)
    try:
        f.serialize(out)
    finally:
        f.setTimeStamp(0)
    bgr, dep, _ = PO.parse_bin(raw)
    assert open(out, "rb").read() == PO.bin_bytes(bgr, dep, ts)
    g = R.Frame360(cal)
    g.loadFrame(out)
    assert g.timeStamp == ts
    g.build(R.BUILD_UNDISTORT | R.BUILD_SPHERE)
    f.build(R.BUILD_UNDISTORT | R.BUILD_SPHERE)
    for a, b in zip(g.sphere(), f.sphere()):
        assert np.array_equal(a, b)


def test_sphere_cloud_matches_oracle(rig):
    for f in rig["frames"]:
        xyz, rgba, w, h = f.sphereCloud()
        xyz4, rgb4, _, _ = f.cloud()
        ox, oc, ow, oh = PO.sphere_cloud(xyz4, rgb4, rig["rt"])
        assert (w, h) == (ow, oh) == (8 * (f.rows // 2), f.cols // 2)
        assert np.array_equal(_bits(xyz), _bits(ox))
        assert np.array_equal(rgba, oc)
        assert np.isfinite(xyz).all(axis=1).mean() > 0.3


def _planes_equal(a, b):
    assert len(a) == len(b)
    for p, q in zip(a, b):
        for k in ("normal", "center", "ppal", "nrgb", "hull"):
            assert np.array_equal(_bits(np.asarray(p[k], np.float32)), _bits(np.asarray(q[k], np.float32))), k
        for k in ("d", "area", "elongation", "curvature", "intensity", "id", "sensor", "n_inliers"):
            assert p[k] == q[k], k


def test_save_and_load_pbmap_cloud(ctx, rig, tmp_path):
    cal, frames = rig["cal"], rig["frames"]
    d = str(tmp_path)
    frames[0].setPlaneLabel(0, "floor")
    for i, f in enumerate(frames):
        f.save(d, i)
    built = [f.planes() for f in frames]
    # the files: PCD bytes = the PCL ascii writer over the oracle sphere cloud; PbMap = the planes
    for i, f in enumerate(frames):
        xyz4, rgb4, _, _ = f.cloud()
        ox, oc, ow, oh = PO.sphere_cloud(xyz4, rgb4, rig["rt"])
        assert open(os.path.join(d, f"sphereCloud_{i}.pcd"), "rb").read() == PO.pcd_bytes(ox, oc, ow, oh, 0)
        filed = PO.pbmap_parse(os.path.join(d, f"spherePlanes_{i}.pbmap"))
        _planes_equal(filed, built[i])
        assert [p["label"] for p in filed][:1] == (["floor"] if i == 0 else [""])
    # a fresh frame restored from the files
    loaded = []
    for i in range(2):
        g = R.Frame360(cal)
        g.load_PbMap_Cloud(d, i)
        _planes_equal(g.planes(), built[i])
        assert g.planeLabel(0) == ("floor" if i == 0 else "")
        xyz, rgba, w, h = g.sphereCloud()
        px, pc, pw, ph = PO.pcd_parse(open(os.path.join(d, f"sphereCloud_{i}.pcd"), "rb").read())
        assert np.array_equal(_bits(xyz), _bits(px)) and np.array_equal(rgba, pc) and (w, h) == (pw, ph)
        loaded.append(g)
    # re-saving a loaded map reproduces the file
    loaded[0].savePlanes(str(tmp_path / "again.pbmap"))
    assert gzip.open(str(tmp_path / "again.pbmap")).read() == gzip.open(os.path.join(d, "spherePlanes_0.pbmap")).read()
    # registration from the loaded maps is the registration of the built ones
    for mode in (R.PLANAR_3DoF, R.DEFAULT_6DoF):
        res = []
        for pair in (frames, loaded):
            reg = R.RegisterRGBD360(ctx)
            ok = reg.RegisterPbMap(pair[0], pair[1], 25, mode)
            res.append((ok, reg.getMatchedPlanes(), reg.getAreaMatched(), reg.getPose().copy(), reg.getInfoMat().copy()))
        assert res[0][:3] == res[1][:3]
        assert np.array_equal(res[0][3], res[1][3]) and np.array_equal(res[0][4], res[1][4])


def test_binary_cloud_modes_and_rebuild(rig, tmp_path):
    cal, f = rig["cal"], rig["frames"][1]
    xyz, rgba, w, h = f.sphereCloud()
    g = R.Frame360(cal)
    for mode in (R.PCD_BINARY, R.PCD_BINARY_COMPRESSED):
        p = str(tmp_path / f"c{mode}.pcd")
        f.saveCloud(p, mode)
        g.loadCloud(p)
        x2, c2, w2, h2 = g.sphereCloud()
        assert np.array_equal(_bits(x2), _bits(xyz)) and np.array_equal(c2, rgba) and (w2, h2) == (w, h)
    # building the frame's cloud replaces the loaded one (buildSphereCloud overwrites sphereCloud)
    g.loadFrame(os.path.join(R.SAMPLES_DIR, SAMPLES[0]))
    g.buildSphereCloud()
    x3, _, _, _ = g.sphereCloud()
    x0, _, _, _ = rig["frames"][0].sphereCloud()
    assert np.array_equal(_bits(x3), _bits(x0))


def test_load_errors(rig, tmp_path):
    g = R.Frame360(rig["cal"])
    with pytest.raises(RuntimeError):
        g.planes()                                   # nothing built or loaded
    with pytest.raises(RuntimeError, match="no sphere cloud"):
        g.sphereCloud()
    bad = str(tmp_path / "bad.pbmap")
    with gzip.open(bad, "wb") as fh:
        fh.write(b"NOTAPBMP" + bytes(8))
    with pytest.raises(RuntimeError, match="not an R360 PbMap"):
        g.loadPbMap(bad)
    rig["frames"][0].savePlanes(bad)
    whole = gzip.open(bad).read()
    with gzip.open(bad, "wb") as fh:
        fh.write(whole[:len(whole) // 2])
    with pytest.raises(RuntimeError, match="truncated|corrupt"):
        g.loadPbMap(bad)
    with pytest.raises(RuntimeError, match="cannot open"):
        g.loadPbMap(str(tmp_path / "missing.pbmap"))
