"""GPU parity tests of RegisterRGBD360::RegisterDensePhotoICP (RegisterRGBD360.h:344-520)
through the C-ABI (r360_register_dense / r360_dense_robot_eval), against oracle/src/robot_oracle.cpp:

* calcPhotoICPError_robot (RegisterPhotoICP.h:4905-5076) + calcHessianGradient_robot (:5083-5407) of all
  8 sensors at fixed poses: identical visible / depth-term counts, error sums to fp64 summation order,
  H / g within 2e-5 of their scale (the reference sums them in float in raster order);
* the full call: the same return value, the pose untouched (the reference's "new" error is evaluated at
  pose_estim), informationM within float-summation tolerance of the oracle's float-serial one;
* edge cases: identical frames (no level runs) and a single valid source pixel (ILL-POSED).
Sizes: the QVGA sample captures (8 x 240 x 320) and a synthetic VGA pair (8 x 480 x 640)."""
import os

import numpy as np
import pytest

import rgbd360_amd as R
from oracle import oracle360 as O

from test_oracle_robot import single_pixel_pair

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return R.Context(0)


def _calib_mats(cal):
    rt, rti, _ = cal.extrinsics()
    return (np.stack([O.from16(rt[16 * k:16 * k + 16]) for k in range(8)]),
            np.stack([O.from16(rti[16 * k:16 * k + 16]) for k in range(8)]))


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
    rt, rti = _calib_mats(cal)
    return dict(cal=cal, frames=frames, raw=raw, rt=rt, rti=rti, rows=240, cols=320)


@pytest.fixture(scope="module")
def vga(ctx):
    cal = R.Calib360(ctx, 480, 640)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    seed = 360 << 16
    A = R.synth_path_pose(seed, 3)
    rel = O.exp_se3([0.0, 0.05, 0.03, np.deg2rad(1.5), 0, 0], pseudo=True).astype(np.float32)
    frames, raw = [], []
    for P in (A, A @ rel):
        b, d = cal.synth_frame(seed, P)
        f = R.Frame360(cal)
        f.upload(b, d)
        f.build(R.BUILD_SENSOR_PYRAMID)
        frames.append(f)
        raw.append((b, d))
    rt, rti = _calib_mats(cal)
    return dict(cal=cal, frames=frames, raw=raw, rt=rt, rti=rti, rows=480, cols=640)


def _poses():
    return [np.eye(4, dtype=np.float32),
            O.exp_se3([0.02, -0.01, 0.03, 0.012, -0.008, 0.01], pseudo=False).astype(np.float32)]


def _eval_check(ctx, D, method, levels):
    f1, f2 = D["frames"]
    (b1, d1), (b2, d2) = D["raw"]
    reg = R.RegisterRGBD360(ctx)
    for l in levels:
        pyr = [(O.sensor_pyramid(b1[k], d1[k], l + 1)[l], O.sensor_pyramid(b2[k], d2[k], l + 1)[l]) for k in range(8)]
        for P in _poses():
            g = reg.eval_dense_robot(f1, f2, l, P, method)
            for k in range(8):
                trg, src = pyr[k]
                e, eP, eD, nv, nd = O.error_robot(src, trg, D["rows"], D["cols"], l, P, D["rt"][k], D["rti"][k],
                                                  method)
                Hf, gf, Hd, gd, nvh = O.hessgrad_robot(src, trg, D["rows"], D["cols"], l, P, D["rt"][k],
                                                       D["rti"][k], method)
                assert (g["n_error"][k], g["n_depth"][k], g["n_vis"][k]) == (nv, nd, nvh), (l, k)
                assert np.isclose(g["err_photo"][k], eP, rtol=1e-9, atol=1e-12), (l, k)
                assert np.isclose(g["err_depth"][k], eD, rtol=1e-9, atol=1e-12), (l, k)
                sc = max(np.abs(Hd).max(), 1e-30)
                assert np.abs(g["H"][k] - Hd).max() <= 2e-5 * sc, (l, k, np.abs(g["H"][k] - Hd).max() / sc)
                sg = max(np.abs(gd).max(), 1e-30)
                assert np.abs(g["g"][k] - gd).max() <= 2e-5 * sg, (l, k)


@pytest.mark.parametrize("method", [R.PHOTO_CONSISTENCY, R.PHOTO_DEPTH, R.DEPTH_CONSISTENCY])
def test_robot_eval_parity_qvga(ctx, qvga, method):
    _eval_check(ctx, qvga, method, (0, 2))


def test_robot_eval_parity_vga(ctx, vga):
    _eval_check(ctx, vga, R.PHOTO_CONSISTENCY, (0, 3))


def _register_check(ctx, D, init, method):
    f1, f2 = D["frames"]
    (b1, d1), (b2, d2) = D["raw"]
    reg = R.RegisterRGBD360(ctx)
    ok = reg.RegisterDensePhotoICP(f1, f2, init, method)
    ook, opose, oinfo, ost = O.register_dense_robot(b1, d1, b2, d2, D["rt"], D["rti"], init, method)
    st = reg.dense_stats
    assert ok == ook
    assert np.array_equal(reg.getPose(), opose) and np.array_equal(opose, init.astype(np.float32))
    assert list(st.ran[:4]) == list(ost.ran[:4]) and st.illposed_level == ost.illposed_level
    for l in range(4):
        assert np.isclose(st.error[l], ost.error[l], rtol=1e-9, atol=1e-12), l
    if ok:
        sc = max(np.abs(oinfo).max(), 1e-30)
        assert np.abs(reg.getInfoMat() - oinfo).max() <= 1e-4 * sc, np.abs(reg.getInfoMat() - oinfo).max() / sc
    return reg, ok


@pytest.mark.parametrize("method", [R.PHOTO_CONSISTENCY, R.PHOTO_DEPTH])
def test_register_dense_parity_qvga(ctx, qvga, method):
    for P in _poses():
        reg, ok = _register_check(ctx, qvga, P, method)
        assert ok and list(reg.dense_stats.ran[:4]) == [1, 1, 1, 1]


def test_register_dense_parity_vga(ctx, vga):
    reg, ok = _register_check(ctx, vga, _poses()[1], R.PHOTO_CONSISTENCY)
    assert ok


def test_register_dense_identical_frames(ctx, qvga):
    f1, _ = qvga["frames"]
    reg = R.RegisterRGBD360(ctx)
    assert reg.RegisterDensePhotoICP(f1, f1, np.eye(4), R.PHOTO_CONSISTENCY)
    st = reg.dense_stats
    assert list(st.ran[:4]) == [0, 0, 0, 0] and st.info_set == 0 and not reg.getInfoMat().any()


def test_register_dense_illposed(ctx):
    cal = R.Calib360(ctx, 48, 64)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    b1, d1, b2, d2 = single_pixel_pair()
    frames = []
    for b, d in ((b1, d1), (b2, d2)):
        f = R.Frame360(cal)
        f.upload(b, d)
        f.build(R.BUILD_SENSOR_PYRAMID)
        frames.append(f)
    rt, rti = _calib_mats(cal)
    init = O.exp_se3([0, 0, 0, np.deg2rad(0.3), 0, 0], pseudo=True).astype(np.float32)
    reg = R.RegisterRGBD360(ctx)
    prev = reg.getInfoMat().copy()
    ok = reg.RegisterDensePhotoICP(frames[0], frames[1], init, R.PHOTO_CONSISTENCY)
    ook, _, _, ost = O.register_dense_robot(b1, d1, b2, d2, rt, rti, init, O.PHOTO)
    assert not ok and not ook
    assert reg.dense_stats.illposed_level == ost.illposed_level == 3
    assert np.array_equal(reg.getPose(), init) and np.array_equal(reg.getInfoMat(), prev)
