"""BASELINE config 5 on one GPU: the 8 x 1280x960 sphere (1280 x 7680 = 9.8 Mpx at level 0, a level-0 working
set above the 256 MB Infinity Cache), with 50 Gauss-Newton iterations at level 0.

Against the CPU oracle on the same synthetic pair (two consecutive frames of the synthetic path):
* stitch and the 5-level pyramid with gradients, bit for bit;
* one fused pass at level 0 (errorPhotoICP_sphere + calcHessGrad_sphere) at two poses: exact counts, H / g to
  1e-5 of scale;
* alignFrames360(PHOTO_DEPTH) with the reference schedule on levels 4..1 and exactly 50 iterations at level 0:
  the pose to the north-star tolerance (1e-4 rad / 1e-3 m), the coarse levels' iteration counts equal;
* three consecutive pairs of the path, and the Register() alias (PbMap-seeded, non-identity start) on one of them;
plus the size-independent properties: source-point compaction counts and the accuracy of the registered
motion against the synthetic ground truth."""
import numpy as np
import pytest

import rgbd360_amd as R
from oracle import oracle360 as O

pytestmark = pytest.mark.gpu

SEED = 360 << 16
ROT_TOL, TRANS_TOL = 1e-4, 1e-3


@pytest.fixture(scope="module")
def hires():
    ctx = R.Context(0)
    cal = R.Calib360(ctx, 960, 1280)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    raw, frames = [], []
    for i in (0, 1, 2, 3):
        b, d = cal.synth_frame(SEED, R.synth_path_pose(SEED, i))
        f = R.Frame360(cal)
        f.upload(b, d)
        f.build()
        raw.append((b, d))
        frames.append(f)
    rt, rti, K = cal.extrinsics()
    return dict(ctx=ctx, cal=cal, frames=frames, raw=raw, rti=rti, K=K.reshape(3, 3).T)


def test_hires_stitch_and_pyramid_bitexact(hires):
    f = hires["frames"][1]
    assert (f.sph_rows, f.sph_cols) == (1280, 7680)
    b, d = hires["raw"][1]
    sb, sd = f.sphere()
    ob, od = O.stitch(b, d, hires["rti"], hires["K"])
    assert np.array_equal(sb, ob) and np.array_equal(sd, od)
    ref = O.sphere_pyramid(sb, sd, 5)
    for l in range(5):
        got = f.level(l)
        for k in ("gray", "depth", "gx", "gy", "dgx", "dgy"):
            assert np.array_equal(got[k], ref[l][k]), (l, k)
        dep = ref[l]["depth"].reshape(-1)
        assert f.points(l).shape[0] == int(((dep > np.float32(0.3)) & (dep < np.float32(6.0))).sum())
    hires["pyr"] = ref


def test_hires_icp_pass_level0(hires):
    f1, f2 = hires["frames"][:2]
    reg = R.RegisterPhotoICP(hires["ctx"])
    reg.setTargetFrame(f1); reg.setSourceFrame(f2)
    lt, ls = f1.level(0), f2.level(0)
    for P in (np.eye(4, dtype=np.float32), O.exp_se3([0.02, -0.03, 0.05, 0.01, -0.015, 0.02])):
        H, g, e2, nv, nvis = reg.eval(0, P, R.PHOTO_DEPTH)
        e, e2r, nvr = O.error_sphere(ls, lt, P, R.PHOTO_DEPTH)
        Hr, gr, nvisr = O.hessgrad_sphere(ls, lt, P, R.PHOTO_DEPTH)
        assert (nv, nvis) == (nvr, nvisr)
        sH = np.abs(Hr).max()
        assert np.abs(H - Hr).max() <= 1e-5 * sH
        scale = np.sqrt(np.abs(np.diag(Hr)) * max(e2r, 1e-30))
        assert (np.abs(g - gr) <= 1e-5 * scale + 1e-12).all()
        assert abs(e2 - e2r) <= 1e-6 * e2r


def _oracle_align(f1, f2, init=None):
    s1b, s1d = f1.sphere()
    s2b, s2d = f2.sphere()
    p = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255), fixed_iters_level0=50)
    return O.align360(s1b, s1d, s2b, s2d, init, O.PHOTO_DEPTH, p)


def _gt_rel(i, j):
    return np.linalg.inv(R.synth_path_pose(SEED, i).astype(np.float64)) @ R.synth_path_pose(SEED, j).astype(np.float64)


def _rot_deg(D):
    return np.degrees(np.arccos(np.clip((np.trace(D[:3, :3]) - 1) / 2, -1, 1)))


@pytest.mark.parametrize("pair", [(1, 2), (2, 3)])
def test_hires_consecutive_pairs(hires, pair):
    """Pairs (1, 2) and (2, 3) of the path (with (0, 1) below: three consecutive pairs), alignFrames360 from identity
    with 50 level-0 iterations, against the oracle; the level-0 pass there streams the packed level-0 images."""
    f1, f2 = (hires["frames"][k] for k in pair)
    reg = R.RegisterPhotoICP(hires["ctx"])
    reg.setNumPyr(5)
    reg.setGrayVariance(3.0 / 255)
    reg.params.fixed_iters_level0 = 50
    reg.setTargetFrame(f1); reg.setSourceFrame(f2)
    rc = reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH)
    rco, pose, H, g, st = _oracle_align(f1, f2)
    assert rc == rco
    assert O.rot_angle(reg.getOptimalPose(), pose) <= ROT_TOL
    assert float(np.linalg.norm(reg.getOptimalPose()[:3, 3] - pose[:3, 3])) <= TRANS_TOL
    assert list(reg.stats.iters)[1:5] == list(st.iters)[1:5]


def test_hires_register_pbmap_seeded(hires):
    """The Register() alias at 8 x 1280x960: PbMap plane extraction of both frames (480 x 640 clouds),
    RegisterPbMap(25, PLANAR_3DoF), the rotOffset-conjugated PbMap pose as alignFrames360's (non-identity)
    initialisation and 50 level-0 iterations, against the oracle's chain on the same raw frames."""
    from rgbd360_amd.odometry import ROT_OFFSET, ROT_OFFSET_INV
    f1, f2 = hires["frames"][2:4]
    p = R.IcpParams.default()
    p.n_pyr = 5
    p.std_dev_photo = np.float32(3.0 / 255)
    p.fixed_iters_level0 = 50
    for f in (f1, f2):
        f.getPlanes()
    pose, info, st, ok = R.register(hires["ctx"], f1, f2, params=p)
    rt, rti, K = hires["cal"].extrinsics()
    rt8 = np.stack([rt[16 * k:16 * k + 16].reshape(4, 4).T for k in range(8)])
    maps = [O.PbMap(d.astype(np.float32) * np.float32(0.001), b, rt8) for (b, d) in hires["raw"][2:4]]
    r = O.register_pbmap(maps[0], maps[1], 25, O.PLANAR_3DoF)
    assert ok == bool(r["good"])
    assert ok, "the synthetic room's planes register"
    assert not np.allclose(r["pose"], np.eye(4), atol=1e-3)          # a non-identity start
    Ro, Ri = ROT_OFFSET.astype(np.float32), ROT_OFFSET_INV.astype(np.float32)
    init = Ro @ r["pose"] @ Ri
    _, dense, _, _, _ = _oracle_align(f1, f2, init)
    ref = Ri.astype(np.float64) @ dense.astype(np.float64) @ Ro.astype(np.float64)
    assert O.rot_angle(pose[:3, :3], ref[:3, :3]) <= ROT_TOL
    assert np.linalg.norm(pose[:3, 3] - ref[:3, 3]) <= TRANS_TOL
    D = np.linalg.inv(_gt_rel(2, 3)) @ pose.astype(np.float64)
    assert _rot_deg(D) < 0.2 and np.linalg.norm(pose[:3, 3] - _gt_rel(2, 3)[:3, 3]) < 0.02


def test_hires_align360_50_iterations(hires):
    f1, f2 = hires["frames"][:2]
    reg = R.RegisterPhotoICP(hires["ctx"])
    reg.setNumPyr(5)
    reg.setGrayVariance(3.0 / 255)
    reg.params.fixed_iters_level0 = 50
    reg.setTargetFrame(f1); reg.setSourceFrame(f2)
    rc = reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH)
    assert reg.stats.passes == sum(1 + reg.stats.evals[l] for l in range(1, 5)) + 1 + 50
    s1b, s1d = f1.sphere()
    s2b, s2d = f2.sphere()
    p = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255), fixed_iters_level0=50)
    rco, pose, H, g, st = O.align360(s1b, s1d, s2b, s2d, None, O.PHOTO_DEPTH, p)
    assert rc == rco
    dr = O.rot_angle(reg.getOptimalPose(), pose)
    dt = float(np.linalg.norm(reg.getOptimalPose()[:3, 3] - pose[:3, 3]))
    assert dr <= ROT_TOL and dt <= TRANS_TOL, (dr, dt)
    assert list(reg.stats.iters)[1:5] == list(st.iters)[1:5]
    # the registered motion is the synthetic path's (sphere frame: rotOffset conjugation)
    from rgbd360_amd.odometry import ROT_OFFSET, ROT_OFFSET_INV
    rig = ROT_OFFSET_INV @ reg.getOptimalPose().astype(np.float64) @ ROT_OFFSET
    gt = np.linalg.inv(R.synth_path_pose(SEED, 0).astype(np.float64)) @ R.synth_path_pose(SEED, 1).astype(np.float64)
    D = np.linalg.inv(gt) @ rig
    assert np.degrees(np.arccos(np.clip((np.trace(D[:3, :3]) - 1) / 2, -1, 1))) < 0.2
    assert np.linalg.norm(rig[:3, 3] - gt[:3, 3]) < 0.02
