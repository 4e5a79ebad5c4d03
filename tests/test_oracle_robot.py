"""CPU checks of the A19 oracle (oracle/src/robot_oracle.cpp): RegisterRGBD360::RegisterDensePhotoICP
(RegisterRGBD360.h:344-520) with calcPhotoICPError_robot (RegisterPhotoICP.h:4905-5076) and
calcHessianGradient_robot (:5083-5407).

* an independent pure-Python restatement of both per-pixel functions (numpy float32 / float64 scalars,
  every cast written out) on a small pyramid level of the reference's sample captures: identical counts,
  the error sums, and the reference's float-serial hessian / gradient bit for bit;
* the level loop: the pose is never moved (the "new" error is evaluated at pose_estim), informationM
  is the float sum of the 8 sensors' level-0 hessians, every level's loop runs on the samples;
* edge cases: identical frames (error 0 -> no level runs, informationM undefined -> zeros) and a
  single valid source pixel (rank-1 Hessian -> ILL-POSED at the coarsest level, false, pose kept).
Parity with the reference itself is unpinned (no reference outputs exist); jacobianRt_z
(uninitialised in the reference, :5372) is taken as zero, which PHOTO_CONSISTENCY never reads."""
import math
import os

import numpy as np
import pytest

from oracle import oracle360 as O

f32, f64 = np.float32, np.float64


@pytest.fixture(scope="module")
def samples(data_dir):
    b1, d1 = O.load_bin(os.path.join(data_dir, "samples", "sphere_images_1.bin"))
    b2, d2 = O.load_bin(os.path.join(data_dir, "samples", "sphere_images_10.bin"))
    rt = O.read_extrinsics(os.path.join(data_dir, "calib", "Extrinsics"))
    rti = np.stack([np.linalg.inv(m.astype(np.float64)).astype(np.float32) for m in rt])
    return b1, d1, b2, d2, rt, rti


def _pose(deg=(1.0, -0.5, 0.7), t=(0.02, -0.01, 0.03)):
    a = np.deg2rad(deg)
    P = O.exp_se3([t[0], t[1], t[2], a[0], a[1], a[2]], pseudo=True)
    return P.astype(np.float32)


def _mv(M, v):  # Eigen Matrix4f * Vector4f: ((m0 x + m1 y) + m2 z) + m3 w, float
    return [f32(f32(f32(f32(M[i, 0] * v[0]) + f32(M[i, 1] * v[1])) + f32(M[i, 2] * v[2])) + f32(M[i, 3] * v[3]))
            for i in range(4)]


def _mm(A, B):  # Eigen Matrix4f product, float, k ascending
    C = np.zeros((4, 4), np.float32)
    for i in range(4):
        for j in range(4):
            s = f32(A[i, 0] * B[0, j])
            for k in range(1, 4):
                s = f32(s + f32(A[i, k] * B[k, j]))
            C[i, j] = s
    return C


def _huber(e, k):
    a = f32(abs(e))
    if a < k:
        return f32(1)
    return f32(f32(math.sqrt(f32(f32(f32(2 * k) * a) - f32(k * k)))) / a)


def _round(x):  # C round(): half away from zero
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def _py_robot(src, trg, rows0, cols0, level, pose, rt, rti, p):
    """Pure-Python calcPhotoICPError_robot + calcHessianGradient_robot (PHOTO_CONSISTENCY)."""
    R, Cn = src["gray"].shape
    w, h = f32(cols0), f32(rows0)
    focal = f32(525 * f32(f64(w) / 640.0))
    ox0, oy0 = f32(f64(w) / 2 - 0.5), f32(f64(h) / 2 - 0.5)
    # error: float intrinsics
    sc = f32(1.0 / 2 ** level)
    fx, ox, oy = f32(focal * sc), f32(ox0 * sc), f32(oy0 * sc)
    ifx = f32(1.0 / f64(fx))
    rel = _mm(_mm(rti, pose), rt)
    # hessgrad: double intrinsics
    scd = 1.0 / 2 ** level
    fxd, oxd, oyd = f64(focal) * scd, f64(ox0) * scd, f64(oy0) * scd
    ifxd = 1.0 / fxd
    sdp = f32(p.std_dev_photo)
    sdp_inv = 1.0 / f64(sdp)
    err, nvis_e = 0.0, 0
    H = np.zeros((6, 6), np.float32)
    g = np.zeros(6, np.float32)
    nvis_h = 0
    for r in range(R):
        for c in range(Cn):
            z = f32(src["depth"][r, c])
            if not (f32(0.3) < z < f32(6.0)):
                continue
            g1 = f32(src["gray"][r, c])
            # ---- error
            x = f32(f32(f32(f32(c) - ox) * z) * ifx)
            y = f32(f32(f32(f32(r) - oy) * z) * ifx)
            tp = _mv(rel, [x, y, z, f32(1)])
            inv = 1.0 / f64(tp[2])
            tc = f64(f32(tp[0] * fx)) * inv + f64(ox)
            tr = f64(f32(tp[1] * fx)) * inv + f64(oy)
            rr, cc = _round(tr), _round(tc)
            if 0 <= rr < R and 0 <= cc < Cn:
                nvis_e += 1
                d = f32(trg["gray"][rr, cc] - g1)
                wp = f64(_huber(d, sdp)) * sdp_inv
                we = f32(wp * f64(d))
                err += f64(f32(we * we))
            # ---- hessgrad
            x = f32(((f64(c) - oxd) * f64(z)) * ifxd)
            y = f32(((f64(r) - oyd) * f64(z)) * ifxd)
            p1 = _mv(rt, [x, y, z, f32(1)])
            p2 = _mv(pose, p1)
            p3 = _mv(rti, p2)
            inv = 1.0 / f64(p3[2])
            tc = (f64(p3[0]) * fxd) * inv + oxd
            tr = (f64(p3[1]) * fxd) * inv + oyd
            rr, cc = _round(tr), _round(tc)
            if not (0 <= rr < R and 0 <= cc < Cn):
                continue
            nvis_h += 1
            gx, gy = f32(trg["gx"][rr, cc]), f32(trg["gy"][rr, cc])
            if abs(gx) < f32(0.01) and abs(gy) < f32(0.01):
                continue
            S = [[f32(1), f32(0), f32(0), f32(0), p2[2], f32(-p2[1])],
                 [f32(0), f32(1), f32(0), f32(-p2[2]), f32(0), p2[0]],
                 [f32(0), f32(0), f32(1), p2[1], f32(-p2[0]), f32(0)]]
            T = [[f32(f32(f32(rti[a, 0] * S[0][b]) + f32(rti[a, 1] * S[1][b])) + f32(rti[a, 2] * S[2][b]))
                  for b in range(6)] for a in range(3)]
            P00, P11 = f32(fxd * inv), f32(fxd * inv)
            P02 = f32(((-fxd * f64(p3[0])) * inv) * inv)
            P12 = f32(((-fxd * f64(p3[1])) * inv) * inv)
            Jw0 = [f32(f32(P00 * T[0][b]) + f32(P02 * T[2][b])) for b in range(6)]
            Jw1 = [f32(f32(P11 * T[1][b]) + f32(P12 * T[2][b])) for b in range(6)]
            d = f32(trg["gray"][rr, cc] - g1)
            wp = f64(_huber(d, sdp)) * sdp_inv
            wf = f32(wp)
            a0, a1 = f32(wf * gx), f32(wf * gy)
            J = [f32(f32(a0 * Jw0[b]) + f32(a1 * Jw1[b])) for b in range(6)]
            res = f32(wp * f64(d))
            for a in range(6):
                for b in range(6):
                    H[a, b] = f32(H[a, b] + f32(J[a] * J[b]))
                g[a] = f32(g[a] + f32(J[a] * res))
    return err, nvis_e, H, g, nvis_h


@pytest.mark.parametrize("sensor", [1, 6])
def test_robot_terms_match_python_restatement(samples, sensor):
    b1, d1, b2, d2, rt, rti = samples
    level = 3
    trg = O.sensor_pyramid(b1[sensor], d1[sensor], level + 1)[level]
    src = O.sensor_pyramid(b2[sensor], d2[sensor], level + 1)[level]
    pose = _pose()
    p = O.IcpParams.default()
    e, eP, eD, nv, nd = O.error_robot(src, trg, 240, 320, level, pose, rt[sensor], rti[sensor], O.PHOTO, p)
    Hf, gf, Hd, gd, nvh = O.hessgrad_robot(src, trg, 240, 320, level, pose, rt[sensor], rti[sensor], O.PHOTO, p)
    pe, pnv, pH, pg, pnvh = _py_robot(src, trg, 240, 320, level, pose, rt[sensor], rti[sensor], p)
    assert nv == pnv and nvh == pnvh and nv > 200
    assert e == eP and nd == 0 and eD == 0.0
    assert e == pe
    assert np.array_equal(Hf.view(np.uint32), pH.T.copy().view(np.uint32))   # symmetric; col-major export
    assert np.array_equal(gf.view(np.uint32), pg.view(np.uint32))
    # the double sums of the same float terms agree with the float-serial ones to float rounding
    scale = np.abs(Hd).max()
    assert np.abs(Hd - Hf).max() <= 1e-4 * scale


def test_register_dense_keeps_pose_and_returns_level0_hessian(samples):
    b1, d1, b2, d2, rt, rti = samples
    p = O.IcpParams.default()
    init = _pose((0.5, 0.2, -0.3), (0.01, 0.0, -0.02))
    ok, pose, info, st = O.register_dense_robot(b1, d1, b2, d2, rt, rti, init, O.PHOTO, p)
    assert ok and np.array_equal(pose, init)
    assert list(st.ran[:4]) == [1, 1, 1, 1] and st.illposed_level == -1 and st.info_set == 1
    assert list(st.iters[:4]) == [0, 0, 0, 0]
    # informationM = sum over sensors (float, in order) of the level-0 float-serial hessians
    Hs = np.zeros((6, 6), np.float32)
    errs = 0.0
    for k in range(8):
        trg = O.sensor_pyramid(b1[k], d1[k], 1)[0]
        src = O.sensor_pyramid(b2[k], d2[k], 1)[0]
        Hf, *_ = O.hessgrad_robot(src, trg, 240, 320, 0, init, rt[k], rti[k], O.PHOTO, p)
        Hs = (Hs + Hf).astype(np.float32)
        errs += O.error_robot(src, trg, 240, 320, 0, init, rt[k], rti[k], O.PHOTO, p)[0]
    assert np.array_equal(info.view(np.uint32), Hs.T.copy().view(np.uint32))
    assert st.error[0] == errs


def test_register_dense_identical_frames_runs_no_level(samples):
    b1, d1, _, _, rt, rti = samples
    ok, pose, info, st = O.register_dense_robot(b1, d1, b1, d1, rt, rti, np.eye(4), O.PHOTO, O.IcpParams.default())
    assert ok and np.array_equal(pose, np.eye(4, dtype=np.float32))
    assert list(st.ran[:4]) == [0, 0, 0, 0] and st.info_set == 0 and not info.any()
    assert all(st.error[l] == 0.0 for l in range(4))


def single_pixel_pair(rows=48, cols=64):
    """frame1: a horizontal ramp on every sensor; frame2: the same ramp darker; all depth invalid but one
    source pixel of sensor 0 (and its target) -> one term per level, a rank-1 Hessian."""
    ramp = np.tile(np.linspace(20, 235, cols).astype(np.uint8)[None, :, None], (rows, 1, 3))
    b1 = np.tile(ramp[None], (8, 1, 1, 1))
    b2 = (b1 // 2).astype(np.uint8)
    d1 = np.zeros((8, rows, cols), np.uint16)
    d2 = np.zeros((8, rows, cols), np.uint16)
    d1[:, :, :] = 1500
    d2[0, rows // 2, cols // 2] = 1500
    return b1, d1, b2, d2


def test_register_dense_illposed_single_region(samples):
    _, _, _, _, rt, rti = samples
    b1, d1, b2, d2 = single_pixel_pair()
    init = _pose((0.3, 0.0, 0.0), (0.0, 0.0, 0.0))
    ok, pose, info, st = O.register_dense_robot(b1, d1, b2, d2, rt, rti, init, O.PHOTO, O.IcpParams.default())
    assert not ok and np.array_equal(pose, init)
    assert st.illposed_level == 3
