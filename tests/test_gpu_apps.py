"""The C++ drivers over the façade (apps/, built by __graft_entry__.build() into build/bin) run end to end on
the GPU and their outputs are checked:
* OdometryRGBD360 (Registration/OdometryRGBD360.cpp loop) on the synthetic path, with and without the
  |t| < 0.4 m frame skip (:230-238): the composed poses against synth_path_pose;
* RegisterPairRGBD360 (config 1) on the reference's sample pair: matched planes and pose equal the oracle's;
* KFsphereTracking (the SLAM/KFsphere_SLAM.cpp tracking calls through the façade): keyframe poses against the
  synthetic ground truth, residual members assigned by the occlusion variant;
* SphereGraphTracking (tracking + loop-closure front end of SLAM/SphereGraphSLAM.cpp over BatchRegistration)."""
import os
import re
import subprocess

import numpy as np
import pytest

import rgbd360_amd as R

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin")
SEED = 360 << 16


def _run(name, *args):
    exe = os.path.join(BIN, name)
    assert os.path.exists(exe), f"{exe} missing: run __graft_entry__.build()"
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr + p.stdout[-2000:]
    return p.stdout


def _gt(k0, k):
    return np.linalg.inv(R.synth_path_pose(SEED, k0).astype(np.float64)) @ R.synth_path_pose(SEED, k).astype(np.float64)


def _pose_err(T, G):
    D = np.linalg.inv(G) @ T
    return np.degrees(np.arccos(np.clip((np.trace(D[:3, :3]) - 1) / 2, -1, 1))), np.linalg.norm(T[:3, 3] - G[:3, 3])


def _poses(out):
    res = {}
    for m in re.finditer(r"pose (\d+):((?: -?\d+\.\d+){12})", out):
        v = np.array([float(x) for x in m.group(2).split()]).reshape(3, 4)
        T = np.eye(4)
        T[:3] = v
        res[int(m.group(1))] = T
    return res


def test_sphere_graph_tracking_synthetic():
    out = _run("SphereGraphTracking", "--synthetic", "10")
    m = re.search(r"(\d+) keyframes, (\d+) loop-closure edges", out)
    assert m, out
    assert int(m.group(1)) == 10                     # every frame of the smooth path tracks
    assert out.count("Good TRACKING") == 9


def test_odometry_synthetic_every_pair():
    out = _run("OdometryRGBD360", "--synthetic", "6")     # frames 1..5 of the path (first = 1), no skip
    assert "5 keyframes" in out and out.count("PbMap ok") == 4, out
    P = _poses(out)
    assert sorted(P) == [2, 3, 4, 5]
    for k, T in P.items():
        dr, dt = _pose_err(T, _gt(1, k))
        assert dr < 0.3 and dt < 0.02, (k, dr, dt)


def test_odometry_synthetic_frame_skip():
    """With the reference's skip, frames closer than 0.4 m to the keyframe are dropped: the path moves
    ~0.1 m per frame, so keyframes are several frames apart, and their composed poses follow the path."""
    out = _run("OdometryRGBD360", "--synthetic", "14", "1")
    P = _poses(out)
    assert 1 <= len(P) < 12, out                       # the skip triggered
    ks = sorted(P)
    assert all(b - a > 1 for a, b in zip([1] + ks, ks)), ks
    for k, T in P.items():                             # >= 0.4 m baselines: a few cm per registration
        dr, dt = _pose_err(T, _gt(1, k))
        path = sum(np.linalg.norm(_gt(j, j + 1)[:3, 3]) for j in range(1, k))
        assert dr < 0.5 and dt < 0.01 + 0.05 * path, (k, dr, dt, path, out)


def test_register_pair_samples_equals_oracle():
    """BASELINE config 1: RegisterPairRGBD360 on samples/sphere_images_1.bin vs _10.bin."""
    from oracle import oracle360 as O
    p1, p2 = (os.path.join(R.SAMPLES_DIR, f"sphere_images_{i}.bin") for i in (1, 10))
    out = _run("RegisterPairRGBD360", p1, p2)
    rt8 = O.read_extrinsics(R.EXTRINSICS_DIR)
    maps = []
    for p in (p1, p2):
        b, d = O.load_bin(p)
        dm = np.stack([O.Clams(os.path.join(R.INTRINSICS_DIR, f"distortion_model{k + 1}.r360")).undistort(
            O.depth_to_m(d[k])) for k in range(8)])
        maps.append(O.PbMap(dm, b, rt8))
    r = O.register_pbmap(maps[0], maps[1], 25, O.PLANAR_3DoF)
    good = "registration good" in out
    assert good == bool(r["good"]), out
    lines = out.split("Pose\n")[0].splitlines()
    matches = {int(a): int(b) for a, b in (l.split() for l in lines if re.fullmatch(r"\d+ \d+", l))}
    assert matches == r["matches"]
    if good:
        pose = np.array([[float(x) for x in l.split()] for l in out.split("Pose\n")[1].strip().splitlines()[:4]])
        np.testing.assert_allclose(pose, r["pose"], atol=2e-6)


def test_kfsphere_tracking_calls():
    """KFsphere_SLAM's tracking calls through the façade (sphere views as setTarget/SourceFrame arguments,
    calcEntropy, trackingScore, occlusion-2 residual members) on the synthetic path."""
    out = _run("KFsphereTracking", "--synthetic", "9", "2")
    assert out.count("PbMap ok") == 8, out
    res = [tuple(float(x) for x in m.groups()) for m in re.finditer(r"Residuals: (\S+) (\S+)", out)]
    assert len(res) == 8 and all(np.isfinite(a) and np.isfinite(b) and a > 0 and b > 0 for a, b in res), res
    ent = [float(m.group(1)) for m in re.finditer(r"entropy (\S+)", out)]
    assert all(np.isfinite(e) for e in ent)
    kf = [(int(m.group(1)), np.array([float(m.group(k)) for k in (2, 3, 4)]))
          for m in re.finditer(r"keyframe (\d+) t = \((\S+) (\S+) (\S+)\)", out)]
    assert kf, out
    for k, t in kf:                                       # keyframe chain vs the path (first frame 0)
        assert np.linalg.norm(t - _gt(0, k)[:3, 3]) < 0.03, (k, t, _gt(0, k)[:3, 3])
    m = re.search(r"(\d+) keyframes", out)
    assert m and int(m.group(1)) == len(kf) + 1
