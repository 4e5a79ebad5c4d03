"""GPU parity tests of the plane half (A3-A9, A11-A13) through the C-ABI, against the CPU oracle on
the same inputs (the two QVGA sample captures with their CLAMS models, and a synthetic VGA pair).

Bars: the per-pixel stages are bit-exact (cloud + median downsample, bilateral filter, normals, CCL
labels, refined labels), the distance map is exact below the 9.5 cap it is consumed at, the per-label
statistics are exact integer moments so plane models, contours, PbMap descriptors, matcher tables,
matches and the PbMap pose are identical to the oracle's.  PCL/MRPT pieces are 'parity unpinned'
against the reference itself."""
import os

import numpy as np
import pytest

import rgbd360_amd as R
from oracle import oracle360 as O

pytestmark = pytest.mark.gpu

def _same(a, b):
    """bitwise equality with NaN == NaN"""
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


@pytest.fixture(scope="module")
def ctx():
    return R.Context(0)


def _oracle_inputs_qvga(path):
    b, d = O.load_bin(path)
    dm = np.stack([O.Clams(os.path.join(R.INTRINSICS_DIR, f"distortion_model{k + 1}.r360")).undistort(O.depth_to_m(d[k]))
                   for k in range(8)])
    return b, dm


@pytest.fixture(scope="module")
def qvga(ctx):
    cal = R.Calib360(ctx, 240, 320)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    cal.loadIntrinsicCalibration(R.INTRINSICS_DIR)
    rt = O.read_extrinsics(R.EXTRINSICS_DIR)
    frames, inputs = [], []
    for name in ("sphere_images_1.bin", "sphere_images_10.bin"):
        p = os.path.join(R.SAMPLES_DIR, name)
        f = R.Frame360(cal)
        f.loadFrame(p)
        f.getPlanes()
        frames.append(f)
        inputs.append(_oracle_inputs_qvga(p))
    return dict(cal=cal, frames=frames, inputs=inputs, rt=rt)


@pytest.fixture(scope="module")
def vga(ctx):
    cal = R.Calib360(ctx, 480, 640)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    rt = O.read_extrinsics(R.EXTRINSICS_DIR)
    seed = 360 << 16
    A = R.synth_path_pose(seed, 0)
    rel = np.eye(4, dtype=np.float32)
    a = np.deg2rad(4.0)
    rel[1:3, 1:3] = [[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]]
    rel[:3, 3] = [0, 0.25, 0.15]
    frames, inputs = [], []
    for P in (A, A @ rel):
        b, d = cal.synth_frame(seed, P)
        f = R.Frame360(cal)
        f.upload(b, d)
        f.getPlanes()
        frames.append(f)
        inputs.append((b, d.astype(np.float32) * np.float32(0.001)))
    return dict(cal=cal, frames=frames, inputs=inputs, rt=rt, rel=rel)


def test_latency_mode_is_result_neutral(vga):
    """The VGA pair on a context with latency mode off (both uploads in stream order, the plane stage launched kernel by
    kernel, PbMap waits on the assembly pool) and rebuilt twice on the default context (the second build replays the
    captured plane-stage graphs): clouds, colours, refined labels and PbMap planes equal the fixture's frames (built
    with latency mode on: split upload, first capture) bit for bit."""
    ctx2 = R.Context(0)
    ctx2.latency_mode(False)
    cal2 = R.Calib360(ctx2, 480, 640)
    cal2.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    seed = 360 << 16
    A = R.synth_path_pose(seed, 0)
    for k, P in enumerate((A, A @ vga["rel"])):
        b, d = vga["cal"].synth_frame(seed, P)
        ref = vga["frames"][k]
        off = R.Frame360(cal2)
        off.upload(b, d)
        off.getPlanes()
        again = R.Frame360(vga["cal"])
        for _ in range(2):
            again.upload(b, d)
            again.getPlanes()
        for f in (off, again):
            for x, y in zip(f.cloud(), ref.cloud()):
                assert _same(x, y)
            for x, y in zip(f.labels(), ref.labels()):
                assert np.array_equal(x, y)
            _cmp_planes(f.planes(), ref.planes())


def _per_sensor_oracle(b, dm):
    out = []
    for k in range(8):
        xyz, rgb = O.cloud_downsample(dm[k], b[k])
        xf = O.bilateral(xyz)
        nrm, dist = O.normals(xf)
        lc, lf, regs = O.segment(xf, nrm)
        out.append(dict(xyz=xf, rgb=rgb, nrm=nrm, dist=dist, lc=lc, lf=lf, regs=regs))
    return out


@pytest.mark.parametrize("which", ["qvga", "vga"])
def test_per_pixel_stages_bitexact(request, which):
    D = request.getfixturevalue(which)
    for f, (b, dm) in zip(D["frames"], D["inputs"]):
        xyz, rgb, nrm, dist = f.cloud()
        lab, labf = f.labels()
        ref = _per_sensor_oracle(b, dm)
        for k in range(8):
            r = ref[k]
            assert _same(xyz[k], r["xyz"]), ("cloud", k)
            assert np.array_equal(rgb[k], r["rgb"]), ("rgb", k)
            assert _same(np.minimum(dist[k], 9.5), np.minimum(r["dist"], 9.5)), ("dist", k)
            assert _same(nrm[k][..., :3], r["nrm"][..., :3]), ("normals", k)
            assert np.array_equal(lab[k], r["lc"]), ("ccl", k)
            assert np.array_equal(labf[k], r["lf"]), ("refined labels", k)
            regs = f.regions(k)
            assert len(regs) == len(r["regs"]), ("regions", k)
            for g, o in zip(regs, r["regs"]):
                assert (g["label"], g["count"], g["start_idx"], g["n_contour"]) == \
                    (o["label"], o["count"], o["start_idx"], len(o["contour"])), ("region", k)
                for key in ("centroid", "cov", "model"):
                    assert np.array_equal(g[key], o[key]), (key, k)
                assert g["curvature"] == o["curvature"]


def _cmp_planes(gp, op):
    assert len(gp) == len(op)
    for g, o in zip(gp, op):
        for key in ("normal", "center", "ppal", "nrgb", "hull"):
            assert np.array_equal(g[key], o[key]), key
        for key in ("d", "area", "elongation", "curvature", "intensity", "id", "sensor", "n_inliers"):
            assert g[key] == o[key], key


@pytest.mark.parametrize("which", ["qvga", "vga"])
def test_pbmap_planes_identical(request, which):
    D = request.getfixturevalue(which)
    maps = []
    for f, (b, dm) in zip(D["frames"], D["inputs"]):
        om = O.PbMap(dm, b, D["rt"])
        _cmp_planes(f.planes(), om.planes())
        maps.append(om)
    D["oracle_maps"] = maps


CONFIG_DIR = os.path.join(R.DATA_DIR, "config_files")


@pytest.mark.parametrize("which", ["qvga", "vga"])
@pytest.mark.parametrize("mode", [R.DEFAULT_6DoF, R.PLANAR_3DoF, R.ODOMETRY_6DoF, R.PLANAR_ODOMETRY_3DoF])
@pytest.mark.parametrize("ini", [None, "configLocaliser_spherical.ini"])
def test_match_tables_and_register_pbmap(ctx, request, which, mode, ini):
    """SubgraphMatcher tables, matches, pose and information for every registrationType
    (RegisterRGBD360.h:260-266), with the default (sphericalOdometry) thresholds and with those of
    configLocaliser_spherical.ini loaded the way RegisterRGBD360(configFile) does (:97-100)."""
    D = request.getfixturevalue(which)
    maps = D.get("oracle_maps") or [O.PbMap(dm, b, D["rt"]) for (b, dm) in D["inputs"]]
    path = os.path.join(CONFIG_DIR, ini) if ini else None
    reg = R.RegisterRGBD360(ctx, path)
    op = O.load_match_ini(path) if path else None
    if op is not None:                       # the two independent ini parsers agree
        assert [getattr(op, f) for f, _ in O.MatchParams._fields_] == [getattr(reg.match, f) for f, _ in R.MatchParams._fields_]
    reg.setReference(D["frames"][0], 25)
    reg.setTarget(D["frames"][1], 25)
    gt = reg.match_tables(mode)
    ot = O.match_tables(maps[0], maps[1], 25, mode, params=op)
    for key in ("sid", "tid", "unary", "binary"):
        assert np.array_equal(gt[key], ot[key]), key
    D.setdefault("tables", {})[(mode, ini)] = ot
    calls0, trunc0, _ = ctx.match_stats()
    ok = reg.RegisterPbMap(D["frames"][0], D["frames"][1], 25, mode)
    r = O.register_pbmap(maps[0], maps[1], 25, mode, params=op)
    calls1, trunc1, max_nodes = ctx.match_stats()
    # the interpretation tree searched to the end (no node-budget cut) on both sides
    assert calls1 == calls0 + 1 and trunc1 == trunc0 and not r["truncated"] and max_nodes >= r["nodes"]
    assert ok == bool(r["good"])
    assert reg.getMatchedPlanes() == r["matches"]
    assert reg.getAreaMatched() == r["area_matched"]
    if ok:
        assert np.array_equal(reg.getPose(), r["pose"])
        assert np.array_equal(reg.getInfoMat(), r["info"])
        # getCovMat / calcEntropy / trackingScore (:208-238, :526-540) from the same information matrix
        cov = np.linalg.inv(r["info"].astype(np.float64))
        np.testing.assert_allclose(reg.getCovMat(), cov, rtol=1e-5, atol=1e-12)
        ent = 0.5 * (6 * (1 + np.log(2 * 3.14159265359)) + np.log(np.linalg.det(cov)))
        assert abs(reg.calcEntropy() - ent) <= 1e-4 * max(1.0, abs(ent))
        q, score = reg.trackingScore()
        assert score == np.float32(np.float32(r["area_matched"]) / np.float32(r["area_src"]))
        assert q == (0 if score >= 0.7 else 1 if score >= 0.3 else 2)


def test_ini_thresholds_change_the_tables(request):
    """configLocaliser_spherical.ini's thresholds (wider area / elongation / distance ratios, other angles)
    give other unary tables than the default file for at least one registrationType, as in the oracle."""
    for which in ("qvga", "vga"):
        T = request.getfixturevalue(which).get("tables", {})
        if not T:
            pytest.skip("runs after test_match_tables_and_register_pbmap")
        diff = [m for m in range(4) if (m, None) in T and (m, "configLocaliser_spherical.ini") in T
                and not np.array_equal(T[(m, None)]["unary"], T[(m, "configLocaliser_spherical.ini")]["unary"])]
        assert diff, which


def test_register_pbmap_synthetic_accuracy(ctx, vga):
    reg = R.RegisterRGBD360(ctx)
    assert reg.RegisterPbMap(vga["frames"][0], vga["frames"][1], 25, R.PLANAR_3DoF)
    P, rel = reg.getPose(), vga["rel"]
    assert np.rad2deg(O.rot_angle(P[:3, :3], rel[:3, :3])) < 0.3
    assert np.linalg.norm(P[:3, 3] - rel[:3, 3]) < 0.02


def _rot_offset(a_deg=157.5):
    """rotOffset of OdometryRGBD360.cpp:138-139 (float angleOffset, double PI) and its transpose."""
    a = np.float64(np.float32(a_deg)) * 3.14159265359 / 180
    Ro = np.eye(4, dtype=np.float32)
    c, s = np.float32(np.cos(a)), np.float32(np.sin(a))
    Ro[1, 1] = Ro[2, 2] = c
    Ro[1, 2], Ro[2, 1] = s, -s
    return Ro, Ro.T.copy()


def _mul4(A, B):
    """Eigen Matrix4f product order in float32: ((a0 b0 + a1 b1) + a2 b2) + a3 b3"""
    C = np.zeros((4, 4), np.float32)
    for r in range(4):
        for c in range(4):
            acc = np.float32(A[r, 0] * B[0, c])
            for k in range(1, 4):
                acc = np.float32(acc + np.float32(A[r, k] * B[k, c]))
            C[r, c] = acc
    return C


def test_register_alias_parity_synth_vga(ctx, vga):
    """Register(): PbMap pose -> rotOffset conjugation -> alignFrames360 (OdometryKeyFrame360.cpp:248-254),
    compared with the oracle chain on the same pair (north-star tolerance 1e-4 rad / 1e-3 m)."""
    f1, f2 = vga["frames"]
    for f in (f1, f2):
        f.build(R.BUILD_UNDISTORT | R.BUILD_SPHERE | R.BUILD_PYRAMID)
    p = R.IcpParams.default()
    p.n_pyr = 5
    p.std_dev_photo = np.float32(3.0 / 255)
    pose, info, st, ok = R.register(ctx, f1, f2, None, p, 25, R.PLANAR_3DoF)
    assert ok
    maps = vga.get("oracle_maps") or [O.PbMap(dm, b, vga["rt"]) for (b, dm) in vga["inputs"]]
    r = O.register_pbmap(maps[0], maps[1], 25, O.PLANAR_3DoF)
    Ro, Ri = _rot_offset()
    init = _mul4(_mul4(Ro, r["pose"]), Ri)
    s1b, s1d = f1.sphere()
    s2b, s2d = f2.sphere()
    op = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255))
    rco, dense, H, g, ost = O.align360(s1b, s1d, s2b, s2d, init, O.PHOTO_DEPTH, op)
    ref = _mul4(_mul4(Ri, dense), Ro)
    assert O.rot_angle(pose[:3, :3], ref[:3, :3]) <= 1e-4
    assert np.linalg.norm(pose[:3, 3] - ref[:3, 3]) <= 1e-3
    # and the registration is right: the synthetic pair's relative pose
    rel = vga["rel"]
    assert np.rad2deg(O.rot_angle(pose[:3, :3], rel[:3, :3])) < 0.2
    assert np.linalg.norm(pose[:3, 3] - rel[:3, 3]) < 0.02


def test_batched_plane_builds_equal_lone_builds(qvga, vga):
    """r360_frames_build: nine synthetic VGA frames (a batch of 8 and a batch of 1) and the two QVGA captures (a
    batch of 2) in one call, frames of two contexts, the batches on the first frame's context stream.  Every frame's
    cloud, normals, labels, PbMap planes and sphere equal its lone build's, and a second batched build of the same
    frames (reused voxel tables and plane buffers) gives them again."""
    ctx2 = R.Context(0)
    calv, calv2 = vga["cal"], R.Calib360(ctx2, 480, 640)
    calv2.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    seed = (360 << 16) + 7
    imgs = [calv.synth_frame(seed, R.synth_path_pose(seed, i)) for i in range(9)]
    flags = R.BUILD_UNDISTORT | R.BUILD_CLOUD | R.BUILD_PLANES | R.BUILD_SPHERE | R.BUILD_PYRAMID
    lone, batch = [], []
    for i, (b, d) in enumerate(imgs):
        f = R.Frame360(calv)
        f.upload(b, d)
        f.build(flags)
        lone.append(f)
        g = R.Frame360(calv2 if i % 2 == 0 else calv)
        g.upload(b, d)
        batch.append(g)
    qb = []
    for name in ("sphere_images_1.bin", "sphere_images_10.bin"):
        g = R.Frame360(qvga["cal"])
        g.loadFrame(os.path.join(R.SAMPLES_DIR, name))
        qb.append(g)
    order = [batch[0], qb[0], *batch[1:5], qb[1], *batch[5:]]
    for rep in range(2):
        R.frames_build(order, flags)
        for g, f in list(zip(batch, lone)) + list(zip(qb, qvga["frames"])):
            for a, b in zip(g.cloud(), f.cloud()):
                assert _same(a, b), rep
            for a, b in zip(g.labels(), f.labels()):
                assert np.array_equal(a, b), rep
            _cmp_planes(g.planes(), f.planes())
        for g, f in zip(batch, lone):
            for a, b in zip(g.sphere(), f.sphere()):
                assert np.array_equal(a, b), rep
