"""GPU tests of the lone-alignment graph cache (r360_align360_async replays its fixed pass sequence as a hipGraph
captured once per pair of frame buffers, host/runtime.cpp align_graph_launch).

The bar is identity with launching the passes one by one: with per-launch timing events on, the ctx takes the
direct path (no graph), so every output of the same alignment (pose, Hessian, gradient, iteration counts, passes,
SSO, error) must be bit-identical between the two paths; and a cache that evicts (more frame pairs than its 8
graphs, frames rebuilt in place between calls) must keep returning the same results as first computed."""
import numpy as np
import pytest

import rgbd360_amd as R

pytestmark = pytest.mark.gpu

SEED = 360 << 16


def _outputs(reg):
    st = reg.stats
    return (reg.getOptimalPose().tobytes(), reg.getHessian().tobytes(), np.asarray(reg.gradient).tobytes(),
            tuple(st.iters), tuple(st.evals), st.passes, st.sso, st.error)


@pytest.fixture(scope="module")
def setup():
    ctx = R.Context(0)
    cal = R.Calib360(ctx, 240, 320)
    cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
    frames = []
    for i in range(5):
        b, d = cal.synth_frame(SEED, R.synth_path_pose(SEED, i))
        f = R.Frame360(cal)
        f.upload(b, d)
        f.build()
        frames.append(f)
    return ctx, frames


def _align(ctx, trg, src, iters0):
    reg = R.RegisterPhotoICP(ctx)
    reg.setNumPyr(4)
    reg.setGrayVariance(3.0 / 255)
    reg.params.fixed_iters_level0 = iters0
    reg.setTargetFrame(trg)
    reg.setSourceFrame(src)
    reg.alignFrames360(np.eye(4), R.PHOTO_DEPTH)
    return _outputs(reg)


@pytest.mark.parametrize("iters0", [0, 10])
def test_graph_replay_equals_direct_launches(setup, iters0):
    ctx, fr = setup
    ctx.timing(True)                 # timing events: passes launched one by one
    direct = _align(ctx, fr[0], fr[1], iters0)
    ctx.timing(False)
    first = _align(ctx, fr[0], fr[1], iters0)    # captured
    again = _align(ctx, fr[0], fr[1], iters0)    # replayed
    assert first == direct
    assert again == direct


def test_graph_cache_eviction_and_rebuilt_frames(setup):
    ctx, fr = setup
    pairs = [(a, b) for a in range(5) for b in range(5) if a != b][:12]   # 12 keys > 8 cached graphs
    ref = {}
    for it in range(2):
        for (a, b) in pairs:
            out = _align(ctx, fr[a], fr[b], 5)
            if it == 0:
                ref[(a, b)] = out
            else:
                assert out == ref[(a, b)], (a, b)
    # a frame rebuilt in place from another image: same buffers, new contents -> the replay reads the new data
    before = _align(ctx, fr[0], fr[4], 5)
    b, d = fr[4].calib.synth_frame(SEED, R.synth_path_pose(SEED, 1))
    fr[4].upload(b, d)
    fr[4].build()
    after = _align(ctx, fr[0], fr[4], 5)
    ctx.timing(True)
    direct = _align(ctx, fr[0], fr[4], 5)
    ctx.timing(False)
    assert after == direct and after != before
