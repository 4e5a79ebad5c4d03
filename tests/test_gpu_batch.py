"""GPU tests of the batched registrations (§8f-4: SphereGraphSLAM tracking, LoopClosure360 candidate checks)
through the C-ABI (r360_batch_register, r360_track_frame).

The bar: a batched job is the single-pair code path run on a worker lane, so every output equals the
sequential call on the same frames — RegisterPbMap (good flag, matches, areas, pose, information) exactly,
and the dense refinement (alignFrames360 after the rotOffset conjugation) to the north-star tolerance of the
sequential Register() chain.  The PbMap stage is also checked against the CPU oracle for the pairs of the
sequence; the tracking winner must be the one the reference's sequential loop picks
(SLAM/SphereGraphSLAM.cpp:175-231)."""
import numpy as np
import pytest

import rgbd360_amd as R
from oracle import oracle360 as O
from test_gpu_planes import _mul4, _rot_offset

pytestmark = pytest.mark.gpu

SEED = 360 << 16
N_FRAMES = 5


@pytest.fixture(scope="module")
def seq():
    """A 5-frame synthetic VGA sequence along the bench's camera path, built on its own ctx (so the
    batch lanes read frames of another stream), plus one frame of an unrelated scene."""
    ctx = R.Context(0)
    cal = R.Calib360(ctx, 480, 640)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    frames, inputs = [], []
    for i in range(N_FRAMES):
        b, d = cal.synth_frame(SEED, R.synth_path_pose(SEED, 2 * i))
        f = R.Frame360(cal)
        f.upload(b, d)
        f.build(R.BUILD_UNDISTORT | R.BUILD_SPHERE | R.BUILD_PYRAMID | R.BUILD_CLOUD | R.BUILD_PLANES)
        frames.append(f)
        inputs.append((b, d.astype(np.float32) * np.float32(0.001)))
    b, d = cal.synth_frame(SEED + 7919, R.synth_path_pose(SEED + 7919, 40))
    other = R.Frame360(cal)
    other.upload(b, d)
    other.build(R.BUILD_UNDISTORT | R.BUILD_SPHERE | R.BUILD_PYRAMID | R.BUILD_CLOUD | R.BUILD_PLANES)
    return dict(ctx=ctx, cal=cal, frames=frames, inputs=inputs, other=other,
                rt=O.read_extrinsics(R.EXTRINSICS_DIR))


@pytest.fixture(scope="module")
def batch():
    return R.Batch(0, lanes=4)


def _seq_pbmap(ctx, ref, trg, mode):
    reg = R.RegisterRGBD360(ctx)
    ok = reg.RegisterPbMap(ref, trg, 25, mode)
    return ok, reg


def _params():
    p = R.IcpParams.default()
    p.n_pyr = 5
    p.std_dev_photo = np.float32(3.0 / 255)
    return p


def test_batch_pbmap_equals_sequential_and_oracle(seq, batch):
    F = seq["frames"] + [seq["other"]]
    pairs = [(F[i], F[j]) for i in range(len(F)) for j in range(len(F)) if i != j]
    res = batch.register_pairs([{"ref": a, "trg": b} for a, b in pairs], 25, R.PLANAR_3DoF)
    ctx = R.Context(0)
    n_good = 0
    for (a, b), r in zip(pairs, res):
        ok, reg = _seq_pbmap(ctx, a, b, R.PLANAR_3DoF)
        assert r["good"] == int(ok)
        assert r["n_match"] == len(reg.getMatchedPlanes())
        assert r["area_matched"] == reg.getAreaMatched()
        assert r["dense_rc"] == -1
        if ok:
            n_good += 1
            assert np.array_equal(r["pbmap_pose"], reg.getPose())
            assert np.array_equal(r["pbmap_info"], reg.getInfoMat())
            assert r["area_src"] == reg.areaSource and r["area_trg"] == reg.areaTarget
            assert r["sso_pbmap"] == np.float32(np.float32(r["area_matched"]) / np.float32(r["area_src"]))
    assert n_good >= N_FRAMES - 1          # consecutive frames of the sequence register
    # the PbMap stage against the CPU oracle on the consecutive pairs
    maps = [O.PbMap(dm, b, seq["rt"]) for (b, dm) in seq["inputs"]]
    for i in range(N_FRAMES - 1):
        o = O.register_pbmap(maps[i], maps[i + 1], 25, O.PLANAR_3DoF)
        k = pairs.index((F[i], F[i + 1]))
        assert res[k]["good"] == int(o["good"])
        assert res[k]["area_matched"] == o["area_matched"]
        if o["good"]:
            assert np.array_equal(res[k]["pbmap_pose"], o["pose"])


def test_track_frame_picks_the_sequential_winner(seq, batch):
    F = seq["frames"]
    ctx = R.Context(0)
    # keyframes oldest first; the newest two are the unrelated frame and a far frame, so the sequential loop
    # may have to walk back
    for kfs, frame in ((F[:3], F[3]), ([F[0], F[1], seq["other"]], F[2]), ([F[0]], F[4]), ([], F[1])):
        chosen, win, cand = batch.track(kfs, frame, num_check=5, no_assoc_threshold=40, max_match_planes=25,
                                        mode=R.PLANAR_ODOMETRY_3DoF)
        assert len(cand) == min(len(kfs), 5)
        # the reference loop (SphereGraphSLAM.cpp:175-231), run sequentially
        expect, expect_reg = -1, None
        for c in range(len(kfs)):
            ok, reg = _seq_pbmap(ctx, kfs[len(kfs) - 1 - c], frame, R.PLANAR_ODOMETRY_3DoF)
            assert cand[c]["good"] == int(ok)
            if ok:
                expect, expect_reg = len(kfs) - 1 - c, reg
                break
        assert chosen == expect
        if expect >= 0:
            assert np.array_equal(win["pbmap_pose"], expect_reg.getPose())
            assert np.array_equal(win["pbmap_info"], expect_reg.getInfoMat())
            assert win["sso_pbmap"] == np.float32(np.float32(expect_reg.getAreaMatched()) /
                                                  np.float32(expect_reg.areaSource))
    # num_check / no_assoc_threshold bound the candidates exactly as the while-condition does
    _, _, cand = batch.track(F[:4], F[4], num_check=2, no_assoc_threshold=40)
    assert len(cand) == 2
    _, _, cand = batch.track(F[:4], F[4], num_check=5, no_assoc_threshold=1)
    assert len(cand) == 1


def test_loop_closure_and_register_jobs_match_sequential(seq, batch):
    F = seq["frames"]
    p = _params()
    ctx = R.Context(0)
    pairs = [(F[0], F[1]), (F[1], F[2]), (F[2], F[3]), (F[0], seq["other"])]
    # Register()-style jobs (dense always, ref = target frame) against r360_register on the same pairs
    jobs = [{"ref": a, "trg": b, "dense": R.JOB_ALWAYS, "ref_is_source": False} for a, b in pairs]
    res = batch.register_pairs(jobs, 25, R.PLANAR_3DoF, params=p)
    for (a, b), r in zip(pairs, res):
        pose, info, st, ok = R.register(ctx, a, b, None, p, 25, R.PLANAR_3DoF)
        assert r["good"] == int(ok) and r["dense_rc"] in (0, 1)
        assert O.rot_angle(r["pose"][:3, :3], pose[:3, :3]) <= 1e-4
        assert np.linalg.norm(r["pose"][:3, 3] - pose[:3, 3]) <= 1e-3
        assert abs(r["sso"] - st.sso) <= 1e-6
    # LoopClosure360 gate (matches > 5, area > 15 m^2) then the refinement with the keyframe as source
    # (LoopClosure360.h:297-313); the gate has to agree with the PbMap outputs, the refinement with a
    # sequential RegisterPhotoICP on the same init
    for mm, ma in ((5, 15.0), (2, 0.0)):
        lc = batch.loop_closures(pairs, min_matches=mm, min_area=ma, ref_is_source=True, params=p)
        for (a, b), r in zip(pairs, lc):
            gate = r["good"] == 1 and r["n_match"] > mm and r["area_matched"] > ma
            assert (r["dense_rc"] >= 0) == gate
            if not gate:
                continue
            Ro, Ri = _rot_offset()
            align = R.RegisterPhotoICP(ctx)
            align.setNumPyr(5)
            align.setGrayVariance(3.0 / 255)
            align.setSourceFrame(a)
            align.setTargetFrame(b)
            align.alignFrames360(_mul4(_mul4(Ro, r["pbmap_pose"]), Ri), R.PHOTO_DEPTH)
            ref = _mul4(_mul4(Ri, align.getOptimalPose()), Ro)
            assert O.rot_angle(r["pose"][:3, :3], ref[:3, :3]) <= 1e-4
            assert np.linalg.norm(r["pose"][:3, 3] - ref[:3, 3]) <= 1e-3
    assert sum(r["dense_rc"] >= 0 for r in lc) >= 3     # relaxed gate: the consecutive pairs are refined


def test_batch_errors_are_loud(seq, batch):
    f = seq["frames"][0]
    with pytest.raises(RuntimeError):
        batch.register_pairs([{"ref": f, "trg": f, "dense": 7}])
