"""CPU oracle checks (no GPU): known-answer tests of each restated primitive against independent
numpy statements, facts the reference's own fixtures fix (samples/*.bin layout and statistics), and
the committed regression fixtures of tests/golden/make_golden.py."""
import hashlib
import os

import numpy as np
import pytest

from oracle import oracle360 as O
from _cases import lambda_family

GOLD = os.path.join(os.path.dirname(__file__), "golden", "oracle_samples.npz")


@pytest.fixture(scope="module")
def samples(data_dir):
    b1, d1 = O.load_bin(os.path.join(data_dir, "samples", "sphere_images_1.bin"))
    b2, d2 = O.load_bin(os.path.join(data_dir, "samples", "sphere_images_10.bin"))
    return b1, d1, b2, d2


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


# ------------------------------------------------------------------ A1: .bin archive
def test_bin_layout_and_statistics(samples):
    b1, d1, _, _ = samples
    assert b1.shape == (8, 240, 320, 3) and d1.shape == (8, 240, 320)
    # measured on this file: channel means (146.8, 164.8, 182.6); 62.6-87.9 % valid depth per sensor
    m = b1.reshape(-1, 3).mean(0)
    assert np.allclose(m, [146.76, 164.79, 182.64], atol=0.01)
    valid = (d1 > 0).reshape(8, -1).mean(1)
    assert valid.min() >= 0.62 and valid.max() <= 0.89
    assert d1.max() <= 9870


def test_bin_writer_reproduces_archive_bytes(tmp_path, data_dir, samples):
    b1, d1, _, _ = samples
    p = str(tmp_path / "x.bin")
    O.write_bin(p, b1, d1)
    src = open(os.path.join(data_dir, "samples", "sphere_images_1.bin"), "rb").read()
    assert open(p, "rb").read() == src


# ------------------------------------------------------------------ A14 primitives
def test_huber_kat():
    assert O.huber(np.float32(0.01), np.float32(0.02)) == 1.0
    e, k = np.float32(0.1), np.float32(0.02)
    exp = np.float32(np.sqrt(np.float32(2 * k * e - k * k))) / e
    assert O.huber(e, k) == np.float32(exp)
    assert O.huber(-e, k) == O.huber(e, k)


def test_rgb2gray_kat():
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [10, 200, 30]]], np.uint8)
    q = px.astype(np.int64)
    y = (q[..., 0] * 4899 + q[..., 1] * 9617 + q[..., 2] * 1868 + 8192) >> 14
    assert list(y[0]) == [76, 150, 29, 124]
    exp = y.astype(np.float32) * np.float32(1.0 / 255)
    assert np.array_equal(O.rgb2gray(px), exp)


def _np_pyrdown(img):
    img = img.astype(np.float32)
    R, C = img.shape
    def refl(p, n):
        p = np.abs(p)
        return np.where(p >= n, 2 * n - p - 2, p)
    xs = 2 * np.arange(C // 2)
    h = (img[:, xs] * np.float32(6) + (img[:, refl(xs - 1, C)] + img[:, refl(xs + 1, C)]) * np.float32(4)
         + img[:, refl(xs - 2, C)] + img[:, refl(xs + 2, C)])
    ys = 2 * np.arange(R // 2)
    r0, r1, r2, r3, r4 = (h[refl(ys + k, R)] for k in (-2, -1, 0, 1, 2))
    t0 = r0 + r4
    t1 = (r1 + r3) + r2
    t0 = t0 + (r2 + r2)
    t0 = t0 + t1 * np.float32(4)
    return t0 * np.float32(1 / 256)


def test_pyrdown_kat():
    rng = np.random.default_rng(0)
    ramp = (np.arange(64, dtype=np.float32).reshape(8, 8) / 63)
    assert np.array_equal(O.pyrdown(ramp), _np_pyrdown(ramp))
    img = rng.random((20, 36), dtype=np.float32)
    assert np.array_equal(O.pyrdown(img), _np_pyrdown(img))


def test_pyr_range_kat():
    d = np.array([[0.0, 1.0, 7.0, 2.0], [0.2, 3.0, 0.5, 0.31]], np.float32)
    out = O.pyr_range(d)
    assert out.shape == (1, 2)
    assert out[0, 0] == np.float32((np.float32(1.0) + np.float32(3.0)) / 2)
    assert out[0, 1] == np.float32((np.float32(2.0) + np.float32(0.5) + np.float32(0.31)) / 3)
    assert O.pyr_range(np.zeros((2, 2), np.float32))[0, 0] == 0


def test_gradient_kat():
    f = np.array([[0, 0, 0], [1, 2, 4], [0, 5, 0]], np.float32)
    gx, gy = O.gradient(f)
    # centre (1,1): 1 < 2 < 4 monotone -> harmonic 2/(1/(4-2) + 1/(2-1)) ; column 0 < 2 < 5
    assert gx[1, 1] == np.float32(2) / (np.float32(1) / np.float32(2) + np.float32(1) / np.float32(1))
    assert gy[1, 1] == np.float32(2) / (np.float32(1) / np.float32(3) + np.float32(1) / np.float32(2))
    assert gx[0, 0] == 0 and gy[2, 1] == 0  # borders
    g2 = np.array([[0, 0, 0], [1, 0, 4], [0, 0, 0]], np.float32)
    assert O.gradient(g2)[0][1, 1] == 0  # not monotone -> 0


def test_exp_se3_kat():
    mu = np.array([0.3, -0.1, 0.2, 0.2, 0.1, -0.3])
    w = mu[3:]
    th = np.linalg.norm(w)
    K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    Rm = np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K
    V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * K + (th - np.sin(th)) / th ** 3 * K @ K
    T = O.exp_se3(mu, True)
    assert np.allclose(T[:3, :3], Rm, atol=1e-7) and np.allclose(T[:3, 3], mu[:3], atol=1e-7)
    T2 = O.exp_se3(mu, False)
    assert np.allclose(T2[:3, 3], V @ mu[:3], atol=1e-6)
    assert np.allclose(O.exp_se3(np.zeros(6)), np.eye(4))


# ------------------------------------------------------------------ A2: CLAMS
def test_clams_interpolated_undistort_kat(data_dir):
    path = os.path.join(data_dir, "calib", "Intrinsics", "distortion_model1.r360")
    raw = open(path, "rb").read()
    hdr = np.frombuffer(raw, np.int32, 7, 11)
    w, h, bw, bh, nx, ny, nb = hdr
    bd = np.frombuffer(raw, np.float64, 1, 11 + 28)[0]
    off = 11 + 36
    counts = np.frombuffer(raw, np.float32, nx * ny * nb, off).reshape(ny, nx, nb)
    mult = np.frombuffer(raw, np.float32, nx * ny * nb, off + 4 * nx * ny * nb).reshape(ny, nx, nb)
    assert (w, h, bw, bh, nx, ny, nb, bd) == (640, 480, 8, 6, 80, 80, 5, 2.0)
    cl = O.Clams(path)
    rng = np.random.default_rng(1)
    z = rng.uniform(0.4, 9.5, (240, 320)).astype(np.float32)
    z[::7, ::5] = 0
    out = cl.undistort(z)
    for (v, u) in [(0, 0), (100, 200), (239, 319), (57, 3), (3, 57)]:
        zz = z[v, u]
        fr_c, fr_m = counts[v // 3, u // 4], mult[v // 3, u // 4]  # downsampleParams(2): 4x3 px bins
        if zz == 0:
            assert out[v, u] == 0
            continue
        idx = min(nb - 1, int(np.floor(zz / bd)))
        start = np.float32(bd * idx)
        idx1 = idx if (zz - start) < bd / 2 else idx + 1
        idx0 = idx1 - 1
        if idx0 < 0 or idx1 >= nb or fr_c[idx0] < 50 or fr_c[idx1] < 50:
            exp = np.float32(zz * fr_m[idx])
        else:
            z0 = (idx0 + 1) * bd - bd * 0.5
            c1 = (float(zz) - z0) / bd
            exp = np.float32(float(zz) * ((1 - c1) * float(fr_m[idx0]) + c1 * float(fr_m[idx1])))
        assert out[v, u] == exp, (v, u)


# ------------------------------------------------------------------ regression fixtures
def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_stitch_and_undistort_golden(samples, gold, data_dir):
    b1, d1, b2, d2 = samples
    s1b, s1d = O.stitch(b1, d1, gold["rti"], gold["K"])
    assert _sha(s1b) + _sha(s1d) == str(gold["sph1_sha"])
    assert s1b.shape == (320, 1920, 3)
    assert 0.7 < (s1d > 0).mean() < 0.9
    cl = [O.Clams(os.path.join(data_dir, "calib", "Intrinsics", f"distortion_model{k + 1}.r360")) for k in range(8)]
    und = np.stack([cl[k].undistort(O.depth_to_m(d1[k])) for k in range(8)])
    assert _sha(und) == str(gold["und1_sha"])


def test_pyramid_and_icp_golden(samples, gold):
    b1, d1, b2, d2 = samples
    s1b, s1d = O.stitch(b1, d1, gold["rti"], gold["K"])
    s2b, s2d = O.stitch(b2, d2, gold["rti"], gold["K"])
    lt, ls = O.sphere_pyramid(s1b, s1d, 5), O.sphere_pyramid(s2b, s2d, 5)
    for l in (3, 4):
        for k in ("gray", "depth", "gx", "gy", "dgx", "dgy"):
            assert np.array_equal(lt[l][k], gold[f"t{l}_{k}"]), (l, k)
            assert np.array_equal(ls[l][k], gold[f"s{l}_{k}"]), (l, k)
        for m in (0, 1, 2):
            for i, P in enumerate(gold["poses"]):
                e, e2, nv = O.error_sphere(ls[l], lt[l], P, m)
                H, g, nvis = O.hessgrad_sphere(ls[l], lt[l], P, m)
                ref = gold[f"icp{l}_{m}_{i}"]
                assert (nv, nvis) == (int(ref[2]), int(ref[3]))
                assert np.allclose([e, e2], ref[:2], rtol=1e-12)
                assert np.allclose(g, ref[4:10], rtol=1e-9, atol=1e-9 * np.abs(ref[4:10]).max())
                assert np.allclose(H.ravel(), ref[10:], rtol=1e-9, atol=1e-9 * np.abs(ref[10:]).max())


def test_align_golden_and_descent(samples, gold):
    b1, d1, b2, d2 = samples
    s1b, s1d = O.stitch(b1, d1, gold["rti"], gold["K"])
    s2b, s2d = O.stitch(b2, d2, gold["rti"], gold["K"])
    p = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255))
    rc, pose, H, g, st = O.align360(s1b, s1d, s2b, s2d, None, O.PHOTO_DEPTH, p)
    assert rc == 0
    assert np.allclose(pose, gold["align_pose"], atol=1e-6)
    assert list(st.iters)[:5] == list(gold["align_iters"])
    # Gauss-Newton descended: the error at the solution is below the error at the initial pose
    lt, ls = O.sphere_pyramid(s1b, s1d, 5), O.sphere_pyramid(s2b, s2d, 5)
    e0 = O.error_sphere(ls[1], lt[1], np.eye(4))[0]
    e1 = O.error_sphere(ls[1], lt[1], pose)[0]
    assert e1 < e0


def _eigen_fullpivlu_rank_f32(M):
    """Independent pure-Python statement of Eigen FullPivLU<Matrix<float,6,6>>::rank() (Eigen 3 FullPivLU.h
    computeInPlace / rank): float arithmetic; the corner's biggest |.| in column-major visiting order (first
    strictly greater, starting at the corner's first coefficient); maxpivot = the largest corner maximum;
    pivots counted above |maxpivot| * (epsilon * 6)."""
    a = [[np.float32(M[r][c]) for c in range(6)] for r in range(6)]
    f = np.float32
    maxpiv, pivs, nz = f(0), [], 6
    for k in range(6):
        br, bc, bv = k, k, abs(a[k][k])
        for c in range(k, 6):
            for r in range(k, 6):
                if (r, c) != (k, k) and abs(a[r][c]) > bv:
                    br, bc, bv = r, c, abs(a[r][c])
        if bv == 0:
            nz = k
            break
        maxpiv = max(maxpiv, bv)
        a[k], a[br] = a[br], a[k]
        for row in a:
            row[k], row[bc] = row[bc], row[k]
        p = a[k][k]
        pivs.append(p)
        for r in range(k + 1, 6):
            a[r][k] = f(a[r][k] / p)
        for r in range(k + 1, 6):
            for c in range(k + 1, 6):
                a[r][c] = f(a[r][c] - f(a[r][k] * a[k][c]))
    thr = f(maxpiv * f(f(1.1920928955078125e-07) * f(6)))
    return sum(1 for k in range(nz) if abs(pivs[k]) > thr)


def test_rank6_is_eigens_float_fullpivlu():
    """The oracle's ILL-POSED test (oracle_la.h rank6) equals an independent statement of Eigen's float
    FullPivLU rank on near-singular matrices, and lambda's decay changes the verdict on some of them."""
    ranks = {}
    for trial, it, M in lambda_family():
        r = O.rank6f(M)
        assert r == _eigen_fullpivlu_rank_f32(M), (trial, it)
        ranks.setdefault(trial, []).append(r)
    flips = [t for t, rs in ranks.items() if rs[0] == 6 and min(rs) < 6]
    assert len(flips) >= 5, ranks          # lambda = 1 passes, a decayed lambda fails
    # singular and zero matrices
    Z = np.zeros((6, 6), np.float32)
    assert O.rank6f(Z) == 0 and _eigen_fullpivlu_rank_f32(Z) == 0
    E = np.eye(6, dtype=np.float32)
    E[5, 5] = 0
    assert O.rank6f(E) == 5 == _eigen_fullpivlu_rank_f32(E)
