"""GPU parity tests of the per-sensor pinhole dense path through the C-ABI,
against oracle/src/pinhole_oracle.cpp on the same inputs:

* RegisterPhotoICP::setSourceFrame / setTargetFrame on each sensor's raw images
  (R360_BUILD_SENSOR_PYRAMID): bit-exact pyramids and gradients, no seam mask;
* errorPhotoICP (:560-761) + calcHessGrad (:767-1100) at fixed poses: exact counts, residual sums to
  fp64 summation order, H / g within 2e-5 of their scale (float accumulation, like the reference's);
* alignFrames (:4254-4512, Levenberg-Marquardt) on all 8 sensors of a pair in one batched launch
  sequence: poses within the north-star bar (1e-4 rad / 1e-3 m) of the oracle's.
Sizes: the two QVGA sample captures (8 x 240 x 320) and a synthetic VGA pair (8 x 480 x 640)."""
import os

import numpy as np
import pytest

import rgbd360_amd as R
from oracle import oracle360 as O

pytestmark = pytest.mark.gpu

METHODS = (R.PHOTO_CONSISTENCY, R.DEPTH_CONSISTENCY, R.PHOTO_DEPTH)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _pose_err(A, B):
    return O.rot_angle(A[:3, :3], B[:3, :3]), float(np.linalg.norm(A[:3, 3] - B[:3, 3]))


@pytest.fixture(scope="module")
def ctx():
    return R.Context(0)


@pytest.fixture(scope="module")
def qvga(ctx):
    cal = R.Calib360(ctx, 240, 320)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    frames, raw = [], []
    for name in ("sphere_images_1.bin", "sphere_images_10.bin"):
        p = os.path.join(R.SAMPLES_DIR, name)
        f = R.Frame360(cal)
        f.loadFrame(p)
        f.build(R.BUILD_SENSOR_PYRAMID)
        frames.append(f)
        raw.append(O.load_bin(p))
    return dict(cal=cal, frames=frames, raw=raw)


@pytest.fixture(scope="module")
def vga(ctx):
    cal = R.Calib360(ctx, 480, 640)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    seed = 360 << 16
    A = R.synth_path_pose(seed, 0)
    rel = np.eye(4, dtype=np.float32)
    a = np.deg2rad(2.0)
    rel[1:3, 1:3] = [[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]]
    rel[:3, 3] = [0, 0.06, 0.04]
    frames, raw = [], []
    for P in (A, A @ rel):
        b, d = cal.synth_frame(seed, P)
        f = R.Frame360(cal)
        f.upload(b, d)
        f.build(R.BUILD_SENSOR_PYRAMID)
        frames.append(f)
        raw.append((b, d))
    return dict(cal=cal, frames=frames, raw=raw, rel=rel, rt=O.read_extrinsics(R.EXTRINSICS_DIR))


def test_sensor_pyramids_bitexact(qvga):
    for f, (b, d) in zip(qvga["frames"], qvga["raw"]):
        for k in (0, 3, 7):
            ref = O.sensor_pyramid(b[k], d[k], 5)
            for l in range(5):
                g = f.sensor_level(k, l)
                for key in ("gray", "depth", "gx", "gy", "dgx", "dgy"):
                    assert np.array_equal(_bits(g[key]), _bits(ref[l][key])), (k, l, key)


def _poses():
    P1 = O.exp_se3([0.01, -0.02, 0.015, 0.01, -0.005, 0.008], pseudo=False)
    P2 = O.exp_se3([-0.05, 0.03, -0.04, -0.02, 0.03, -0.01], pseudo=False)
    return [np.eye(4, dtype=np.float32), P1, P2]


@pytest.mark.parametrize("method", METHODS)
def test_eval_parity(ctx, qvga, method):
    f_t, f_s = qvga["frames"]
    (bt, dt), (bs, ds) = qvga["raw"]
    reg = R.RegisterPhotoICP(ctx)
    K = O.Pinhole.rgbd360(240, 320)
    for k in (0, 5):
        reg.setTargetSensor(f_t, k)
        reg.setSourceSensor(f_s, k)
        pt, ps = O.sensor_pyramid(bt[k], dt[k], 4), O.sensor_pyramid(bs[k], ds[k], 4)
        for l in (0, 2):
            for P in _poses():
                g = reg.eval_pinhole(l, P, method)
                e, nP, nD, rP, rD = O.error_pinhole(ps[l], pt[l], K, l, P, method)
                H, gg, nvis = O.hessgrad_pinhole(ps[l], pt[l], K, l, P, method)
                assert (g["n_photo"], g["n_depth"], g["n_vis"]) == (nP, nD, nvis), (k, l)
                assert np.isclose(g["res_photo"], rP, rtol=1e-9, atol=0) and np.isclose(g["res_depth"], rD, rtol=1e-9,
                                                                                         atol=0)
                if method == R.PHOTO_CONSISTENCY:
                    assert np.isnan(g["error"]) and np.isnan(e)   # avPhoto divides by nValidDepthPts (:760)
                else:
                    assert np.isclose(g["error"], e, rtol=1e-9, atol=0)
                sc = max(np.abs(H).max(), 1e-30)
                assert np.abs(g["H"] - H).max() <= 2e-5 * sc, (k, l, np.abs(g["H"] - H).max() / sc)
                sg = max(np.abs(gg).max(), 1e-30)
                assert np.abs(g["g"] - gg).max() <= 2e-5 * sg, (k, l)


def _align_all(ctx, D, inits, method, n_pyr):
    f_t, f_s = D["frames"]
    reg = R.RegisterPhotoICP(ctx)
    reg.setNumPyr(n_pyr)
    poses, Hs, stats, ill = reg.alignSensors(f_t, f_s, list(range(8)), inits, method)
    (bt, dt), (bs, ds) = D["raw"]
    p = O.IcpParams.default(n_pyr=n_pyr)
    ref = [O.align_pinhole(bt[k], dt[k], bs[k], ds[k], init=inits[k], method=method, params=p) for k in range(8)]
    return reg, poses, Hs, stats, ill, ref


def _oracle_stable(D, k, init, method, n_pyr, ref_pose):
    """Whether the oracle's own solve of sensor k is stable under a rounding-level perturbation of the
    initial pose (1e-7 rad about x, about one float ulp): the perturbed solve must stay inside the
    parity bar itself.  On the real captures some sensors slide down a poorly
    constrained valley for 40 iterations (e.g. sensor 5 drifts 0.32 m with PHOTO_DEPTH), where the
    float accumulation order alone (the reference's omp critical sums, :1080-1097) changes the
    outcome; parity is asserted on the sensors where the reference's answer is itself well defined."""
    (bt, dt), (bs, ds) = D["raw"]
    tweak = O.exp_se3([0, 0, 0, 1e-7, 0, 0], pseudo=False).astype(np.float32)
    p = O.IcpParams.default(n_pyr=n_pyr)
    _, Pp, _, _, stp = O.align_pinhole(bt[k], dt[k], bs[k], ds[k], init=(tweak @ init).astype(np.float32),
                                       method=method, params=p)
    dr, dtr = _pose_err(Pp, ref_pose)
    return dr <= 1e-4 and dtr <= 1e-3, dr, dtr, stp.error


@pytest.mark.parametrize("method", [R.PHOTO_DEPTH, R.DEPTH_CONSISTENCY])
def test_align_sensors_parity_qvga(ctx, qvga, method):
    inits = [np.eye(4, dtype=np.float32)] * 8
    reg, poses, Hs, stats, ill, ref = _align_all(ctx, qvga, inits, method, 4)
    checked = 0
    for k in range(8):
        rc, Po, Ho, go, st = ref[k]
        assert stats[k].illposed == rc
        stable, sdr, sdt, serr = _oracle_stable(qvga, k, inits[k], method, 4, Po)
        dr, dtr = _pose_err(poses[k], Po)
        if not stable:
            # the reference's own answer moves by (sdr, sdt) under a 1e-7 rad nudge of the initial pose (a flat
            # valley), so the pose is not comparable; the solve must still reach the same quality: its final
            # error within 2 % of the oracle's, or within twice the oracle's own change under the nudge (a solve
            # that regressed still fails)
            tol = max(0.02 * abs(st.error), 2 * abs(serr - st.error))
            assert abs(stats[k].error - st.error) <= tol, (k, stats[k].error, st.error, serr, sdr, sdt)
            continue
        checked += 1
        assert dr <= 1e-4 and dtr <= 1e-3, (k, dr, dtr, list(stats[k].iters[:4]), list(st.iters[:4]))
        # the residual members alignFrames leaves (:4329-4332, :4507-4509; errorPhotoICP :759-762)
        assert stats[k].residuals_set == st.residuals_set, k
        if st.residuals_set:
            for a, b in ((stats[k].av_photo_residual, st.av_photo_residual),
                         (stats[k].av_depth_residual, st.av_depth_residual), (stats[k].av_residual, st.av_residual)):
                # at poses equal to the north-star tolerance: 1e-3 relative
                assert (np.isnan(a) and np.isnan(b)) or abs(a - b) <= 1e-3 * abs(b), (k, a, b)
    assert checked >= 5, checked
    # the single-sensor entry point is the same computation
    f_t, f_s = qvga["frames"]
    reg.setTargetSensor(f_t, 3)
    reg.setSourceSensor(f_s, 3)
    reg.alignFrames(inits[3], method)
    assert np.array_equal(reg.getOptimalPose(), poses[3])
    assert np.array_equal(reg.getHessian(), Hs[3])


def test_photo_only_never_iterates(ctx, qvga):
    """errorPhotoICP's PHOTO_CONSISTENCY value is NaN (:760), so the LM loop never starts (:4324)."""
    P = _poses()[1]
    reg, poses, Hs, stats, ill, ref = _align_all(ctx, qvga, [P] * 8, R.PHOTO_CONSISTENCY, 3)
    for k in range(8):
        assert np.array_equal(poses[k], P) and np.array_equal(ref[k][1], P)
        assert list(stats[k].iters[:3]) == [0, 0, 0] == list(ref[k][4].iters[:3])


def test_align_sensors_synthetic_vga(ctx, vga):
    """Sensor-frame motion of the rig motion rel: Rt_k^-1 rel Rt_k (MethodsRegisterRGBD360.cpp:336).
    Parity with the oracle, and the solve recovers the motion on the textured synthetic room."""
    rt = vga["rt"]
    truth = [np.linalg.inv(rt[k].astype(np.float64)) @ vga["rel"] @ rt[k] for k in range(8)]
    inits = [np.eye(4, dtype=np.float32)] * 8
    reg, poses, Hs, stats, ill, ref = _align_all(ctx, vga, inits, R.PHOTO_DEPTH, 5)
    assert ill == 0
    good = 0
    for k in range(8):
        dr, dtr = _pose_err(poses[k], ref[k][1])
        assert dr <= 1e-4 and dtr <= 1e-3, (k, dr, dtr)
        er, et = _pose_err(poses[k], truth[k])
        good += (er < np.deg2rad(0.5) and et < 0.02)
    assert good == 8, good
