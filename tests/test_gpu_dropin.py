"""Source-level drop-in: tests/dropin/odometry_dropin.cpp is the reference's OdometryRGBD360
call sequence (Registration/OdometryRGBD360.cpp:60-257) compiled against include/rgbd360/compat.h with the
reference's own constructors — Calib360 calib (QVGA), default-argument calibration loads, RegisterRGBD360(ini),
RegisterPhotoICP align360 — and built by __graft_entry__.build() into build/bin.  Run on the reference's sample pair
(sphere_images_1.bin -> _10.bin, selectSample 9), its RegisterPbMap verdict / matched pose and its alignFrames360
pose must equal the CPU oracle's on the same inputs (north-star tolerance for the dense pose)."""
import os
import re
import subprocess

import numpy as np
import pytest

import rgbd360_amd as R

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "bin", "odometry_dropin")


def _pose(out, tag):
    m = re.search(re.escape(tag) + r":((?: \S+){16})", out)
    assert m, (tag, out)
    return np.array([float(x) for x in m.group(1).split()]).reshape(4, 4)


def test_odometry_call_sequence_on_samples_equals_oracle():
    from oracle import oracle360 as O
    assert os.path.exists(EXE), f"{EXE} missing: run __graft_entry__.build()"
    p = subprocess.run([EXE, R.SAMPLES_DIR, "1", "9"], capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr + p.stdout[-2000:]
    out = p.stdout
    assert "1 registrations" in out, out

    p1, p2 = (os.path.join(R.SAMPLES_DIR, f"sphere_images_{i}.bin") for i in (1, 10))
    (b1, d1), (b2, d2) = O.load_bin(p1), O.load_bin(p2)
    # PbMap stage: RegisterPbMap(frame360_1, frame360_2, 25, PLANAR_3DoF) (:166)
    rt8 = O.read_extrinsics(R.EXTRINSICS_DIR)
    maps = []
    for b, d in ((b1, d1), (b2, d2)):
        dm = np.stack([O.Clams(os.path.join(R.INTRINSICS_DIR, f"distortion_model{k + 1}.r360")).undistort(
            O.depth_to_m(d[k])) for k in range(8)])
        maps.append(O.PbMap(dm, b, rt8))
    r = O.register_pbmap(maps[0], maps[1], 25, O.PLANAR_3DoF)
    good = "pbmap good:" in out
    assert good == bool(r["good"]), out
    if good:
        np.testing.assert_allclose(_pose(out, "pbmap good"), r["pose"], atol=2e-6)
    # dense stage: alignFrames360(Identity, PHOTO_DEPTH) on the stitched spheres (:189-193), QVGA calibration
    ctx = R.Context(0)
    cal = R.Calib360(ctx, 240, 320)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    _, rti, K = cal.extrinsics()
    Km = K.reshape(3, 3).T
    s1b, s1d = O.stitch(b1, d1, rti, Km)
    s2b, s2d = O.stitch(b2, d2, rti, Km)
    prm = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255))
    _, opose, _, _, _ = O.align360(s1b, s1d, s2b, s2d, None, O.PHOTO_DEPTH, prm)
    dense = _pose(out, "dense optimal")
    assert O.rot_angle(dense, opose) <= 1e-4 and np.linalg.norm(dense[:3, 3] - opose[:3, 3]) <= 1e-3, (dense, opose)
