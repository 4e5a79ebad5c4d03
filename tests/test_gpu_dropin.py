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


SG_EXE = os.path.join(ROOT, "build", "bin", "sphere_graph_dropin")


def _lines(out, tag):
    return [ln[len(tag):] for ln in out.splitlines() if ln.startswith(tag)]


def test_sphere_graph_and_loop_closure_call_sites(tmp_path):
    """tests/dropin/sphere_graph_dropin.cpp over three synthetic captures of the benchmark's path at the samples'
    QVGA size, written as the reference's .bin archives (the two sample captures are too far apart for the
    odometry modes' unary constraints: the tracking loop finds no association): SphereGraphSLAM's tracking on the
    main thread (RegisterPbMap PLANAR_ODOMETRY_3DoF, getPose / getInfoMat into Eigen::Matrix<float,6,6>,
    getAreaMatched() / areaSource) and LoopClosure360's keyframe registration on a second std::thread over frames the
    main thread built (RegisterPbMap PLANAR_3DoF, then alignFrames360 of the keyframe spheres, stitched on first use
    from that thread).  Bars: the PbMap stages equal the oracle's, the dense pose is within the north-star tolerance
    of the oracle's, the loop thread's output equals the same calls made on the main thread, and a frame built on
    the loop thread's own default context registers after that thread has exited."""
    from oracle import oracle360 as O
    from rgbd360_amd import odometry as OD
    assert os.path.exists(SG_EXE), f"{SG_EXE} missing: run __graft_entry__.build()"
    seed = 360 << 16
    rt8 = O.read_extrinsics(R.EXTRINSICS_DIR)
    caps = []
    for k in range(3):
        b, d = R.synth_frame_rt(240, 320, rt8, seed, R.synth_path_pose(seed, k))
        O.write_bin(str(tmp_path / f"sphere_images_{k + 1}.bin"), b, d)
        caps.append((b, d))
    p = subprocess.run([SG_EXE, str(tmp_path), "1", "1"], capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr + p.stdout[-3000:]
    out = p.stdout
    assert "2 tracked" in out and "lc error" not in out, out

    maps = []
    for b, d in caps:
        dm = np.stack([O.Clams(os.path.join(R.INTRINSICS_DIR, f"distortion_model{k + 1}.r360")).undistort(
            O.depth_to_m(d[k])) for k in range(8)])
        maps.append(O.PbMap(dm, b, rt8))

    def mats(tag, n):
        return [np.array([float(x) for x in ln.split()]).reshape(n, n) for ln in _lines(out, tag + ":")]

    # tracking (:175-201): each new frame against the newest keyframe
    poses, infos = mats("track pose", 4), mats("track info", 6)
    ssos = [float(x) for x in re.findall(r"track SSO (\S+)", out)]
    for k in range(2):
        tr = O.register_pbmap(maps[k], maps[k + 1], 25, O.PLANAR_ODOMETRY_3DoF)
        assert tr["good"] == 1, k
        np.testing.assert_allclose(poses[k], tr["pose"], atol=2e-6)
        np.testing.assert_allclose(infos[k], tr["info"], rtol=1e-6, atol=1e-6)
        assert abs(ssos[k] - np.float32(tr["area_matched"]) / np.float32(tr["area_src"])) <= 1e-6
    # the frame built on the exited loop thread (the third capture) against the first keyframe
    lt = O.register_pbmap(maps[0], maps[2], 25, O.PLANAR_ODOMETRY_3DoF)
    assert int(re.search(r"lt pbmap good (\d)", out).group(1)) == lt["good"]
    if lt["good"]:
        np.testing.assert_allclose(_pose(out, "lt pbmap pose"), lt["pose"], atol=2e-6)
    # loop closure (:297-314): PLANAR_3DoF, then the dense refinement of the keyframe spheres
    lc = O.register_pbmap(maps[0], maps[1], 25, O.PLANAR_3DoF)
    m = re.search(r"lc pbmap good (\d) matches (\d+)", out)
    assert int(m.group(1)) == lc["good"] == 1 and int(m.group(2)) == len(lc["matches"])
    np.testing.assert_allclose(_pose(out, "lc pbmap pose"), lc["pose"], atol=2e-6)
    ctx = R.Context(0)
    cal = R.Calib360(ctx, 240, 320)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    _, rti, K = cal.extrinsics()
    Km = K.reshape(3, 3).T
    (s1b, s1d), (s2b, s2d) = (O.stitch(b, d, rti, Km) for b, d in caps[:2])
    Ro, Ri = OD.ROT_OFFSET.astype(np.float32), OD.ROT_OFFSET_INV.astype(np.float32)
    rel = _pose(out, "lc pbmap pose").astype(np.float32)
    init = (Ro @ rel @ Ri).astype(np.float32)
    prm = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255))
    _, opose, _, _, _ = O.align360(s2b, s2d, s1b, s1d, init, O.PHOTO_DEPTH, prm)   # target newKF, source keyframe
    ref = Ri.astype(np.float64) @ opose.astype(np.float64) @ Ro.astype(np.float64)
    dense = _pose(out, "lc dense pose")
    assert O.rot_angle(dense, ref) <= 1e-4 and np.linalg.norm(dense[:3, 3] - ref[:3, 3]) <= 1e-3, (dense, ref)
    # cross-thread == same-thread, line for line
    for tag in (" pbmap good", " pbmap pose:", " pbmap info:", " dense pose:", " dense hessian:", " dense SSO"):
        assert _lines(out, "lc" + tag) == _lines(out, "st" + tag) and _lines(out, "lc" + tag), tag
