"""BASELINE config 5 on one GPU: the 8 x 1280x960 sphere (1280 x 7680 = 9.8 Mpx at level 0, a level-0 working
set above the 256 MB Infinity Cache), with 50 Gauss-Newton iterations at level 0.

Against the CPU oracle on the same synthetic pair (two consecutive frames of the synthetic path):
* stitch and the 5-level pyramid with gradients, bit for bit;
* one fused pass at level 0 (errorPhotoICP_sphere + calcHessGrad_sphere) at two poses: exact counts, H / g to
  1e-5 of scale;
* alignFrames360(PHOTO_DEPTH) with the reference schedule on levels 4..1 and exactly 50 iterations at level 0:
  the pose to the north-star tolerance (1e-4 rad / 1e-3 m), the coarse levels' iteration counts equal;
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
    for i in (0, 1):
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
    f1, f2 = hires["frames"]
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


def test_hires_align360_50_iterations(hires):
    f1, f2 = hires["frames"]
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
