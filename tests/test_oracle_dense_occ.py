"""CPU checks of the oracle's occlusion-aware restatement (RegisterPhotoICP.h:3232-4250) on a small
synthetic sphere level: structural properties that follow from the reference's code."""
import numpy as np

from oracle import oracle360 as O


def _level(rows, cols, seed):
    rng = np.random.default_rng(seed)
    r = np.arange(rows)[:, None]
    c = np.arange(cols)[None, :]
    gray = (0.5 + 0.4 * np.sin(c * 0.21) * np.cos(r * 0.17) + 0.05 * rng.random((rows, cols))).astype(np.float32)
    depth = (2.0 + 0.8 * np.sin(c * 0.05) + 0.3 * np.cos(r * 0.11)).astype(np.float32)
    holes = rng.random((rows, cols)) < 0.05
    gx = np.zeros_like(gray); gy = np.zeros_like(gray)
    dgx = np.zeros_like(gray); dgy = np.zeros_like(gray)
    gx[:, 1:-1] = (gray[:, 2:] - gray[:, :-2]) / 2
    gy[1:-1, :] = (gray[2:, :] - gray[:-2, :]) / 2
    dgx[:, 1:-1] = (depth[:, 2:] - depth[:, :-2]) / 2
    dgy[1:-1, :] = (depth[2:, :] - depth[:-2, :]) / 2
    depth[holes] = np.nan                 # no target depth: not finite, excluded from the depth terms
    dgx[holes] = dgy[holes] = 0.0
    return dict(gray=gray, depth=depth, gx=gx, gy=gy, dgx=dgx, dgy=dgy)


def test_occ1_hessgrad_is_plain_and_occ2_bounded():
    src, trg = _level(40, 240, 1), _level(40, 240, 2)
    P = O.exp_se3([0.3, -0.2, 0.25, 0.05, -0.04, 0.06])
    H0, g0, n0 = O.hessgrad_sphere(src, trg, P, O.PHOTO_DEPTH)
    H1, g1, n1 = O.hessgrad_sphere_occ(src, trg, P, O.PHOTO_DEPTH, 1)
    # (the plain function merges its OpenMP partial sums in arrival order: equal to fp64 rounding)
    assert n1 == n0 and np.allclose(H1, H0, rtol=1e-12, atol=0) and np.allclose(g1, g0, rtol=1e-12, atol=1e-9)
    H2, g2, n2 = O.hessgrad_sphere_occ(src, trg, P, O.PHOTO_DEPTH, 2)
    assert 0 < n2 <= n0                      # at most one point per target pixel, outliers dropped
    e0, _, nv0 = O.error_sphere(src, trg, P, O.PHOTO_DEPTH)
    e1, nv1 = O.error_sphere_occ(src, trg, P, O.PHOTO_DEPTH, 1)
    e2, nv2 = O.error_sphere_occ(src, trg, P, O.PHOTO_DEPTH, 2)
    assert 0 < nv1 <= nv0 and 0 < nv2 <= n0
    assert np.isfinite(e1) and np.isfinite(e2)
    # occlusion 0 through the dispatcher is the plain error (OpenMP merge order: fp64 rounding)
    assert np.isclose(O.error_sphere_occ(src, trg, P, O.PHOTO_DEPTH, 0)[0], e0, rtol=1e-13, atol=0)


def test_occ1_photo_only_has_no_depth_terms():
    """errorPhotoICP_sphereOcc1 returns avPhoto + avDepth with avDepth = sqrt(0 / 0) when no depth term
    is evaluated (PHOTO_CONSISTENCY): the reference's value is NaN."""
    src, trg = _level(20, 120, 3), _level(20, 120, 4)
    e, nv = O.error_sphere_occ(src, trg, np.eye(4, dtype=np.float32), O.PHOTO, 1)
    assert np.isnan(e) and nv > 0
