"""GPU parity tests of the dense half of the hot path (run on an MI355X through gpurun):
undistort, stitch, pyramids/gradients, the fused ICP pass and alignFrames360, all through the C-ABI,
compared with the CPU oracle on the same inputs.

Bars: integer/byte outputs and the deterministic float pipelines (stitch, gray, pyramids,
gradients, CLAMS) are bit-exact; the ICP sums differ only by fp64 summation order and rare 1-ulp
asinf/atan2f rounding flips (glibc vs ocml), so H/g/err2 are checked to 1e-5 relative and the counts
to 1e-4 of the pixels; poses to the north-star tolerance 1e-4 rad / 1e-3 m."""
import os

import numpy as np
import pytest

import rgbd360_amd as R
from oracle import oracle360 as O

pytestmark = pytest.mark.gpu

ROT_TOL, TRANS_TOL = 1e-4, 1e-3


@pytest.fixture(scope="module")
def ctx():
    # no explicit close: frames/calibs hold the ctx alive and are destroyed first
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
    b1, d1 = O.load_bin(os.path.join(R.SAMPLES_DIR, "sphere_images_1.bin"))
    b2, d2 = O.load_bin(os.path.join(R.SAMPLES_DIR, "sphere_images_10.bin"))
    rt, rti, K = cal.extrinsics()
    Km = K.reshape(3, 3).T
    return dict(cal=cal, f1=f1, f2=f2, raw=(b1, d1, b2, d2), rti=rti, K=Km)


def _pose_err(A, B):
    return O.rot_angle(A, B), float(np.linalg.norm(np.asarray(A)[:3, 3] - np.asarray(B)[:3, 3]))


def test_libm_port_bitexact_on_device():
    """The device asinf/atan2f (libm_f32.h) equals glibc's std::asin/std::atan2 bit for bit."""
    rng = np.random.default_rng(7)
    n = 1 << 22
    x = rng.uniform(-1, 1, n).astype(np.float32)
    y = rng.uniform(-6, 6, n).astype(np.float32)
    z = rng.uniform(-6, 6, n).astype(np.float32)
    a, t = R.libm_eval(x, y, z, on_device=True)
    ra, rt = O.libm(x, y, z)
    # bit-equal, except that any NaN matches any NaN (payload/sign are not part of the contract)
    for u, v in ((a, ra), (t, rt)):
        same = (u.view(np.uint32) == v.view(np.uint32)) | (np.isnan(u) & np.isnan(v))
        assert same.all(), np.flatnonzero(~same)[:10]


def test_undistort_bitexact(qvga):
    b1, d1, _, _ = qvga["raw"]
    gpu = qvga["f1"].depth_m()
    for k in range(8):
        cl = O.Clams(os.path.join(R.INTRINSICS_DIR, f"distortion_model{k + 1}.r360"))
        ref = cl.undistort(O.depth_to_m(d1[k]))
        assert np.array_equal(gpu[k], ref), k


def test_stitch_bitexact(qvga):
    b1, d1, b2, d2 = qvga["raw"]
    for f, b, d in ((qvga["f1"], b1, d1), (qvga["f2"], b2, d2)):
        gb, gd = f.sphere()
        ob, od = O.stitch(b, d, qvga["rti"], qvga["K"])
        assert np.array_equal(gb, ob)
        assert np.array_equal(gd, od)


def test_pyramid_bitexact(qvga):
    for f in (qvga["f1"], qvga["f2"]):
        sb, sd = f.sphere()
        ref = O.sphere_pyramid(sb, sd, 6)
        for l in range(6):
            got = f.level(l)
            for k in ("gray", "depth", "gx", "gy", "dgx", "dgy"):
                assert np.array_equal(got[k], ref[l][k]), (l, k)


def test_source_points_compaction(qvga):
    """The ICP pass streams each level's valid source pixels (0.3 < depth < 6, RegisterPhotoICP.h:4578) as
    compacted {LUT point, gray} records in raster order (frame_kernels.hip k_src_*): same count, same gray
    values in the same order, and LUT points at the pixel's depth along its viewing ray."""
    for f in (qvga["f1"], qvga["f2"]):
        for l in range(6):
            lv = f.level(l)
            d, gray = lv["depth"].reshape(-1), lv["gray"].reshape(-1)
            valid = (d > np.float32(0.3)) & (d < np.float32(6.0))
            pts = f.points(l)
            assert pts.shape[0] == int(valid.sum()), l
            assert np.array_equal(pts[:, 3], gray[valid]), l
            np.testing.assert_allclose(np.linalg.norm(pts[:, :3].astype(np.float64), axis=1), d[valid], rtol=2e-6)
            rows, cols = lv["depth"].shape
            r, c = np.nonzero(valid.reshape(rows, cols))
            ares = 2 * np.pi / cols
            phi = (rows / 2 - 0.5 - r) * ares
            np.testing.assert_allclose(pts[:, 0], d[valid] * np.sin(phi), atol=2e-5)


def _icp_check(H, g, e2, nv, nvis, Hr, gr, e2r, nvr, nvisr, npx):
    """The projection is bit-identical (glibc-exact asinf/atan2f port), so pixel sets and counts
    match exactly; the sums differ only by summation order (GPU: per-thread f32 partials over a few
    pixels, then fp64), bounded per component by 1e-5 of the Cauchy-Schwarz scale sqrt(H_kk e2)."""
    assert (nv, nvis) == (nvr, nvisr)
    sH = np.abs(Hr).max()
    assert np.abs(H - Hr).max() <= 1e-5 * sH
    scale = np.sqrt(np.abs(np.diag(Hr)) * max(e2r, 1e-30))
    assert (np.abs(g - gr) <= 1e-5 * scale + 1e-12).all(), (g - gr, scale)
    assert abs(e2 - e2r) <= 1e-6 * e2r


@pytest.mark.parametrize("method", [0, 1, 2])
def test_icp_pass_parity_samples(ctx, qvga, method):
    reg = R.RegisterPhotoICP(ctx)
    reg.setTargetFrame(qvga["f1"]); reg.setSourceFrame(qvga["f2"])
    poses = [np.eye(4, dtype=np.float32), O.exp_se3([0.02, -0.03, 0.05, 0.01, -0.015, 0.02])]
    for l in range(5):
        lt, ls = qvga["f1"].level(l), qvga["f2"].level(l)
        for P in poses:
            H, g, e2, nv, nvis = reg.eval(l, P, method)
            e, e2r, nvr = O.error_sphere(ls, lt, P, method)
            Hr, gr, nvisr = O.hessgrad_sphere(ls, lt, P, method)
            _icp_check(H, g, e2, nv, nvis, Hr, gr, e2r, nvr, nvisr, lt["gray"].size)


@pytest.mark.parametrize("method", [0, 1, 2])
def test_icp_image_stream_pass_parity_samples(ctx, qvga, method):
    """The pass forms of batched launches over frames without compacted source points (r360_frame_set_compaction 0:
    the sequence runner's ring frames): the level's image streamed as PF 6 at level 0 (packed), PF 8 where rows split
    into whole waves (960 columns) and PF 9 where a wave spans two rows (480 / 240 / 120 columns); sums, counts and
    errors against the oracle at every level with the bars of the compacted form."""
    cal = qvga["cal"]
    f1, f2 = R.Frame360(cal), R.Frame360(cal)
    for f, k in ((f1, 0), (f2, 2)):
        b, d = qvga["raw"][k], qvga["raw"][k + 1]
        f.setCompaction(False)
        f.upload(b, d)
        f.build()
    reg = R.RegisterPhotoICP(ctx)
    reg.setTargetFrame(f1); reg.setSourceFrame(f2)
    poses = [np.eye(4, dtype=np.float32), O.exp_se3([0.02, -0.03, 0.05, 0.01, -0.015, 0.02])]
    for l in range(5):
        lt, ls = f1.level(l), f2.level(l)
        for P in poses:
            H, g, e2, nv, nvis = reg.eval(l, P, method)
            e, e2r, nvr = O.error_sphere(ls, lt, P, method)
            Hr, gr, nvisr = O.hessgrad_sphere(ls, lt, P, method)
            _icp_check(H, g, e2, nv, nvis, Hr, gr, e2r, nvr, nvisr, lt["gray"].size)
    # compacted on request, as before
    pts = f2.points(2)
    d = f2.level(2)["depth"].reshape(-1)
    assert pts.shape[0] == int(((d > np.float32(0.3)) & (d < np.float32(6.0))).sum())


def test_align360_parity_samples(ctx, qvga):
    reg = R.RegisterPhotoICP(ctx)
    reg.setNumPyr(5); reg.setGrayVariance(3.0 / 255)           # Registration/OdometryRGBD360.cpp:92-95
    reg.setTargetFrame(qvga["f1"]); reg.setSourceFrame(qvga["f2"])
    rc = reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH)
    b1, d1, b2, d2 = qvga["raw"]
    s1b, s1d = O.stitch(b1, d1, qvga["rti"], qvga["K"])
    s2b, s2d = O.stitch(b2, d2, qvga["rti"], qvga["K"])
    p = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255))
    rco, pose, H, g, st = O.align360(s1b, s1d, s2b, s2d, None, O.PHOTO_DEPTH, p)
    assert rc == rco
    dr, dt = _pose_err(reg.getOptimalPose(), pose)
    assert dr <= ROT_TOL and dt <= TRANS_TOL, (dr, dt)
    assert list(reg.stats.iters)[:5] == list(st.iters)[:5]
    # H is evaluated at the final pose; poses agree to ~1e-7, which can move a handful of pixels across
    # a rounding boundary of the projection, so H agrees to ~1e-4 of its scale, not bit for bit
    assert np.allclose(reg.getHessian(), H, rtol=2e-3, atol=2e-3 * np.abs(H).max())


@pytest.fixture(scope="module")
def vga(ctx):
    cal = R.Calib360(ctx, 480, 640)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    seed = 360 << 16
    A = R.synth_path_pose(seed, 0)
    rel = np.eye(4, dtype=np.float32)
    a = np.deg2rad(4.0)
    rel[1:3, 1:3] = [[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]]
    rel[:3, 3] = [0, 0.25, 0.15]
    B = A @ rel
    b1, d1 = cal.synth_frame(seed, A)
    b2, d2 = cal.synth_frame(seed, B)
    f1, f2 = R.Frame360(cal), R.Frame360(cal)
    f1.upload(b1, d1); f2.upload(b2, d2)
    f1.build(); f2.build()
    rt, rti, K = cal.extrinsics()
    return dict(cal=cal, f1=f1, f2=f2, raw=(b1, d1, b2, d2), rti=rti, K=K.reshape(3, 3).T, rel=rel)


def test_synth_frame_statistics(vga):
    b1, d1, b2, d2 = vga["raw"]
    hole = (d1 == 0).reshape(8, -1).mean(1)
    assert (hole > 0.05).all() and (hole < 0.45).all(), hole
    assert d1[d1 > 0].min() >= 400 and d1.max() <= 8000


@pytest.mark.parametrize("fixed", [0, 20])
def test_align360_parity_synth_vga(ctx, vga, fixed):
    reg = R.RegisterPhotoICP(ctx)
    reg.setNumPyr(5); reg.setGrayVariance(3.0 / 255)
    reg.params.fixed_iters_level0 = fixed
    reg.setTargetFrame(vga["f1"]); reg.setSourceFrame(vga["f2"])
    rc = reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH)
    b1, d1, b2, d2 = vga["raw"]
    s1b, s1d = vga["f1"].sphere()
    s2b, s2d = vga["f2"].sphere()
    ob, od = O.stitch(b1, d1, vga["rti"], vga["K"])
    assert np.array_equal(ob, s1b) and np.array_equal(od, s1d)
    p = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255), fixed_iters_level0=fixed)
    rco, pose, H, g, st = O.align360(s1b, s1d, s2b, s2d, None, O.PHOTO_DEPTH, p)
    assert rc == rco
    dr, dt = _pose_err(reg.getOptimalPose(), pose)
    assert dr <= ROT_TOL and dt <= TRANS_TOL, (dr, dt)
    if fixed:
        assert reg.stats.passes == sum(1 + st.evals[l] for l in range(1, 5)) + 1 + fixed


@pytest.mark.parametrize("rows,cols", [(640, 3840), (320, 1920), (160, 960), (40, 240), (960, 3840), (1920, 3840)])
def test_fast_projection_guard_never_changes_a_pixel(rows, cols):
    """The pass projects with hardware rsq/rcp and falls back to the exact (reference) program inside a
    guard band around every .5 rounding boundary; over random and boundary-adversarial points the pass's
    decisions (visible or not, and which target pixel) must be identical to the exact program's.  (Near the
    poles, far outside the 60-degree band, the fast row can differ by more than the guard; such points are
    invisible either way.)  The last two geometries are spheres taller than the stitched one (H = W / 4 and
    W / 2, r360_calib_create_sphere): rows beyond 32 degrees are in view there, and the fast asin defers
    them to the exact projection instead of placing them outside."""
    rng = np.random.default_rng(rows * 7 + cols)
    n = 1 << 22
    # directions over the whole sphere, ranges 0.2-12 m
    v = rng.normal(size=(n, 3)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    v *= rng.uniform(0.2, 12.0, size=(n, 1)).astype(np.float32)
    # adversarial: directions placed on pixel-rounding boundaries of this geometry (+- a few ulps)
    m = n // 4
    ares = 2 * 3.14159265359 / cols
    r = rng.integers(-2, rows + 2, m) + 0.5 + rng.normal(scale=1e-4, size=m)
    c = rng.integers(-2, cols + 2, m) + 0.5 + rng.normal(scale=1e-4, size=m)
    phi = (rows / 2 - 0.5 - r) * ares
    th = c * ares - 3.14159265359
    d = rng.uniform(0.3, 8.0, m)
    v[:m, 0] = d * np.sin(phi)
    v[:m, 1] = d * np.cos(phi) * np.sin(th)
    v[:m, 2] = d * np.cos(phi) * np.cos(th)
    x, y, z = (np.ascontiguousarray(v[:, k]) for k in range(3))
    mism, fb = R.C.c_ulonglong(), R.C.c_ulonglong()
    R._check(R.lib().r360_proj_check(R._fptr(x), R._fptr(y), R._fptr(z), n, rows, cols, R.C.byref(mism),
                                     R.C.byref(fb)), "proj_check")
    assert mism.value == 0, mism.value
    fb_cap = n // 3 if rows * 6 <= cols else (2 * n) // 3   # tall spheres: |x| >= 0.53 always deferred
    assert fb.value < fb_cap          # the fast path decides most points
    # the same with a pose: LUT points whose TRANSFORMED position is random or on a rounding boundary,
    # so the fast (FMA-contracted) transform is covered too
    for seed in range(3):
        P = O.exp_se3(rng.normal(scale=[0.2, 0.2, 0.2, 0.1, 0.1, 0.1]), pseudo=False).astype(np.float32)
        lut = ((v - P[:3, 3]) @ P[:3, :3]).astype(np.float32)   # R^T (p' - t)
        lx, ly, lz = (np.ascontiguousarray(lut[:, k]) for k in range(3))
        p16 = np.ascontiguousarray(P.T).reshape(16)
        R._check(R.lib().r360_proj_check_pose(R._fptr(lx), R._fptr(ly), R._fptr(lz), n, R._fptr(p16), rows, cols,
                                              R.C.byref(mism), R.C.byref(fb)), "proj_check_pose")
        assert mism.value == 0, (seed, mism.value)
        assert fb.value < fb_cap


def test_correctly_rounded_sqrt_div():
    """The pass's error terms use sqrt_rn / div_rn (libm_f32.h): they must equal IEEE sqrtf and '/' bit for
    bit over the operand ranges the pass feeds them (64M operands each)."""
    out = (R.C.c_ulonglong * 2)()
    R._check(R.lib().r360_rn_check(1 << 26, 7, out), "rn_check")
    assert out[0] == 0 and out[1] == 0, (out[0], out[1])


def test_rank_test_matches_oracle_over_lambda_schedule():
    """The device ILL-POSED tests (icp_la.inc rank6_rows of the GN step and wave_rank6 of the pinhole / robot steps:
    Eigen's float FullPivLU rank; r360_rank6 returns -1 where the two disagree) give the oracle's verdict on
    near-singular Hessians over alignFrames360's decaying lambda (1, /5 per accepted update, RegisterPhotoICP.h:4589,
    :4718), including the ones where the decay flips it."""
    from _cases import lambda_family
    fam = lambda_family()
    M = np.ascontiguousarray(np.stack([m for _, _, m in fam]), np.float32)
    out = np.zeros(len(fam), np.int32)
    R._check(R.lib().r360_rank6(R._fptr(M), len(fam), out.ctypes.data_as(R.C.POINTER(R.C.c_int))), "rank6")
    ref = np.array([O.rank6f(m) for _, _, m in fam])
    assert np.array_equal(out, ref)
    assert (ref < 6).any() and (ref == 6).any()


def test_gn_solve_matches_oracle():
    """The GN step's solve (icp_la.inc solve6_rows_dpp: row per lane, DPP pivot search) gives the
    oracle's x = -H^-1 g (oracle_la.h solve6) bit for bit: SPD Hessians of the scales the passes produce, badly
    conditioned ones, and matrices whose pivot order differs from the diagonal's."""
    rng = np.random.default_rng(7)
    Hs, gs = [], []
    for k in range(256):
        J = rng.normal(size=(6, 40)) * (10.0 ** rng.uniform(-3, 3, size=(6, 1)))
        H = (J @ J.T).astype(np.float32).astype(np.float64)   # the passes' H / g are float sums
        if k % 4 == 1:
            H = rng.normal(size=(6, 6)).astype(np.float32).astype(np.float64)   # non-symmetric: row swaps
        if k % 4 == 2:
            H[5] = H[4] * (1 + 1e-6)                                          # nearly singular
        Hs.append(H)
        gs.append(rng.normal(size=6).astype(np.float32).astype(np.float64) * 10.0 ** rng.uniform(-3, 3))
    H = np.ascontiguousarray(np.stack(Hs))
    g = np.ascontiguousarray(np.stack(gs))
    x = np.zeros((len(Hs), 6))
    R._check(R.lib().r360_solve6(R._dptr(H), R._dptr(g), len(Hs), R._dptr(x)), "solve6")
    ref = [O.solve6(h, gg) for h, gg in zip(Hs, gs)]
    ok = [k for k, r in enumerate(ref) if r is not None]     # exactly singular systems: no oracle answer
    assert len(ok) > 240
    assert np.array_equal(x[ok].view(np.uint64), np.stack([ref[k] for k in ok]).view(np.uint64))


def test_set_frames_from_sphere_images(ctx, qvga):
    """setSourceFrame / setTargetFrame(imgRGB, imgDepth) (RegisterPhotoICP.h:480-516): the stitched spheres
    handed over as images (downloaded, then uploaded into sphere-only frames) give the same pyramid and the
    same alignment as the frames themselves."""
    f1, f2 = qvga["f1"], qvga["f2"]
    s1b, s1d = f1.sphere()
    s2b, s2d = f2.sphere()
    a = R.RegisterPhotoICP(ctx)
    b = R.RegisterPhotoICP(ctx)
    for reg in (a, b):
        reg.setNumPyr(5)
        reg.setGrayVariance(3.0 / 255)
    a.setTargetFrame(f1); a.setSourceFrame(f2)
    b.setTargetFrame(s1b, s1d); b.setSourceFrame(s2b, s2d)
    for l in range(5):
        la, lb = f2.level(l), b.src.level(l)
        for k in ("gray", "depth", "gx", "gy", "dgx", "dgy"):
            assert np.array_equal(la[k], lb[k]), (l, k)
        assert np.array_equal(f2.points(l), b.src.points(l)), l
    ra = a.alignFrames360(np.eye(4), R.PHOTO_DEPTH)
    rb = b.alignFrames360(np.eye(4), R.PHOTO_DEPTH)
    assert ra == rb
    assert np.array_equal(a.getOptimalPose(), b.getOptimalPose())
    assert np.array_equal(a.getHessian(), b.getHessian())
