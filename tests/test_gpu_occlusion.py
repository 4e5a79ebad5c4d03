"""GPU parity of the occlusion-aware dense variants: errorPhotoICP_sphereOcc1/2,
calcHessGrad_sphereOcc2 and alignFrames360(occlusion = 1 / 2), through the C-ABI, against the CPU
oracle's sequential restatement (RegisterPhotoICP.h:3232-4250, :4598-4627).

The reference runs these loops under OpenMP with unsynchronised Z-buffer writes; the oracle and the GPU
both take the LUT order (source index ascending), so the accepted point sets, counts and visible counts
are identical and the sums differ only by summation order."""
import os

import numpy as np
import pytest

import rgbd360_amd as R
from oracle import oracle360 as O

pytestmark = pytest.mark.gpu

ROT_TOL, TRANS_TOL = 1e-4, 1e-3


@pytest.fixture(scope="module")
def ctx():
    return R.Context(0)


@pytest.fixture(scope="module")
def qvga(ctx):
    cal = R.Calib360(ctx, 240, 320)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    cal.loadIntrinsicCalibration(R.INTRINSICS_DIR)
    f1, f2 = R.Frame360(cal), R.Frame360(cal)
    f1.loadFrame(os.path.join(R.SAMPLES_DIR, "sphere_images_1.bin"))
    f2.loadFrame(os.path.join(R.SAMPLES_DIR, "sphere_images_10.bin"))
    f1.build(); f2.build()
    return dict(cal=cal, f1=f1, f2=f2)


def _close(a, b, rel):
    if np.isnan(a) or np.isnan(b):
        return np.isnan(a) and np.isnan(b)
    return abs(a - b) <= rel * abs(b)


POSES = [np.eye(4, dtype=np.float32), O.exp_se3([0.02, -0.03, 0.05, 0.01, -0.015, 0.02]),
         O.exp_se3([-0.15, 0.1, -0.2, 0.03, 0.02, -0.04])]


@pytest.mark.parametrize("occ", [1, 2])
@pytest.mark.parametrize("method", [0, 1, 2])
def test_occlusion_pass_parity(ctx, qvga, method, occ):
    reg = R.RegisterPhotoICP(ctx)
    reg.setTargetFrame(qvga["f1"]); reg.setSourceFrame(qvga["f2"])
    for l in range(5):
        lt, ls = qvga["f1"].level(l), qvga["f2"].level(l)
        for P in POSES:
            H, g, e, nv, nvis = reg.eval_occ(l, P, method, occ)
            er, nvr = O.error_sphere_occ(ls, lt, P, method, occ)
            Hr, gr, nvisr = O.hessgrad_sphere_occ(ls, lt, P, method, occ)
            assert (nv, nvis) == (nvr, nvisr), (l, nv, nvr, nvis, nvisr)
            assert _close(e, er, 1e-6), (l, e, er)
            sH = max(np.abs(Hr).max(), 1e-30)
            assert np.abs(H - Hr).max() <= 1e-5 * sH
            scale = np.sqrt(np.abs(np.diag(Hr)) * sH) + 1e-12
            assert (np.abs(g - gr) <= 1e-5 * scale).all(), (g - gr, scale)


def test_occ1_hessgrad_equals_plain(ctx, qvga):
    """calcHessGrad_sphereOcc1 indexes its Z-buffer by the source pixel (:3486-3488), so it never
    occludes: its H / g / numVisiblePixels are calcHessGrad_sphere's.  (The plain pass streams the compacted
    source points, the occlusion pass the image, so the f32 partial sums group pixels differently: equal
    counts, sums equal to summation-order rounding.)"""
    reg = R.RegisterPhotoICP(ctx)
    reg.setTargetFrame(qvga["f1"]); reg.setSourceFrame(qvga["f2"])
    P = POSES[1]
    H1, g1, _, _, nvis1 = reg.eval_occ(1, P, R.PHOTO_DEPTH, 1)
    H0, g0, _, _, nvis0 = reg.eval(1, P, R.PHOTO_DEPTH)
    assert nvis1 == nvis0
    sH = np.abs(H0).max()
    assert np.abs(H1 - H0).max() <= 1e-6 * sH
    assert (np.abs(g1 - g0) <= 1e-6 * np.sqrt(np.abs(np.diag(H0)) * sH)).all()


def test_occ2_filters_and_occludes(ctx, qvga):
    """Occ2 keeps at most one point per target pixel for H / g and drops depth outliers: fewer visible
    pixels than the plain pass, and every count is bounded by the plain one."""
    reg = R.RegisterPhotoICP(ctx)
    reg.setTargetFrame(qvga["f1"]); reg.setSourceFrame(qvga["f2"])
    P = POSES[2]
    _, _, _, nv2, nvis2 = reg.eval_occ(0, P, R.PHOTO_DEPTH, 2)
    _, _, _, nv0, nvis0 = reg.eval(0, P, R.PHOTO_DEPTH)
    assert 0 < nvis2 < nvis0
    assert 0 < nv2 <= nvis0


@pytest.mark.parametrize("occ", [1, 2])
def test_align360_occlusion_parity_samples(ctx, qvga, occ):
    reg = R.RegisterPhotoICP(ctx)
    reg.setNumPyr(5); reg.setGrayVariance(3.0 / 255)
    reg.setTargetFrame(qvga["f1"]); reg.setSourceFrame(qvga["f2"])
    rc = reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH, occ)
    s1b, s1d = qvga["f1"].sphere()
    s2b, s2d = qvga["f2"].sphere()
    p = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255))
    rco, pose, H, g, st = O.align360(s1b, s1d, s2b, s2d, None, O.PHOTO_DEPTH, p, occlusion=occ)
    assert rc == rco
    dr = O.rot_angle(reg.getOptimalPose(), pose)
    dt = float(np.linalg.norm(np.asarray(reg.getOptimalPose())[:3, 3] - pose[:3, 3]))
    assert dr <= ROT_TOL and dt <= TRANS_TOL, (dr, dt)
    assert list(reg.stats.iters)[:5] == list(st.iters)[:5]
    # the residual members errorPhotoICP_sphereOcc1/2 leave (RegisterPhotoICP.h:3360-3362, :3852-3853)
    assert reg.stats.residuals_set & 1 and st.residuals_set & 1
    # evaluated at the final poses, which agree to the north-star tolerance (not bit for bit): 1e-3 relative
    assert _close(reg.avPhotoResidual, st.av_photo_residual, 1e-3), (reg.avPhotoResidual, st.av_photo_residual)
    assert _close(reg.avDepthResidual, st.av_depth_residual, 1e-3), (reg.avDepthResidual, st.av_depth_residual)
    assert (reg.stats.residuals_set & 2) == (st.residuals_set & 2)        # avResidual only when ILL-POSED


def test_plain_align_leaves_residual_members(ctx, qvga):
    """errorPhotoICP_sphere assigns no residual member: after an occlusion-0 alignment they keep the values
    of the previous occlusion-2 one (uninitialised in a fresh reference object: NaN here)."""
    reg = R.RegisterPhotoICP(ctx)
    reg.setNumPyr(4)
    reg.setTargetFrame(qvga["f1"]); reg.setSourceFrame(qvga["f2"])
    reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH, 0)
    assert np.isnan(reg.avPhotoResidual) and np.isnan(reg.avDepthResidual) and np.isnan(reg.avResidual)
    reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH, 2)
    a, b = reg.avPhotoResidual, reg.avDepthResidual
    assert np.isfinite(a) and np.isfinite(b)
    reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH, 0)
    assert (reg.avPhotoResidual, reg.avDepthResidual) == (a, b)
