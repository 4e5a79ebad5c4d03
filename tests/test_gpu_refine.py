"""GPU tests of the banded refinement sweeps (k_refine_p1 / k_refine_p2): OrganizedMultiPlaneSegmentation's
refine() (restated in oracle/src/planes_oracle.cpp) as two raster sweeps whose row-to-row
dependency is resolved by speculative row bands plus an in-order fix-up.

The bar: bit-identical swept states to the sequential sweep, for every band height, on inputs built to make
labels travel far across band boundaries (large non-planar regions whose pixels are close to several
models), against
  * a pure-Python restatement of the two sweeps (small sensors), and
  * the single-wave sweep kernel (rb = 0; bit-exact against the CPU oracle end to end in test_gpu_planes.py)
    at the bench's 320 x 240 sensors and at HiRes width.
The end-to-end plane tests (test_gpu_planes.py) run the banded sweeps by default."""
import numpy as np
import pytest

import rgbd360_amd as R

pytestmark = pytest.mark.gpu


def _refine_ref(S, M):
    """The two sweeps of one sensor, sequentially (state -1 none, -2 non-planar, m >= 0 planar model m)."""
    S = S.astype(np.int64).copy()
    h, w = S.shape

    def close(m, v):
        return (int(m) >> int(v)) & 1

    for r in range(h - 1):                      # first sweep: rows 0..h-2, left to right, right/down checks
        L = S[r].copy()
        F = L.copy()
        v = -2
        for c in range(w):
            F[c] = v if (L[c] == -2 and v >= 0 and close(M[r, c], v)) else L[c]
            v = F[c]
        for c in range(w - 1):
            if F[c] == -1 or L[c + 1] == -1 or S[r + 1, c] == -1:
                continue
            if F[c] >= 0 and S[r + 1, c] == -2 and close(M[r + 1, c], F[c]):
                S[r + 1, c] = F[c]
        S[r] = F
    for r in range(h - 1, 0, -1):               # second sweep: rows h-1..1, right to left, left/up checks
        L = S[r].copy()
        F = L.copy()
        v = -2
        for c in range(w - 1, -1, -1):
            F[c] = v if (L[c] == -2 and v >= 0 and close(M[r, c], v)) else L[c]
            v = F[c]
        for c in range(w - 1, 0, -1):
            if F[c] == -1 or L[c - 1] == -1 or S[r - 1, c] == -1:
                continue
            if F[c] >= 0 and S[r - 1, c] == -2 and close(M[r - 1, c], F[c]):
                S[r - 1, c] = F[c]
        # column 0: its "left" neighbour is the last pixel of the row above (flat-index wrap)
        upw, upw_m, f0, up0, um0 = S[r - 1, w - 1], M[r - 1, w - 1], F[0], S[r - 1, 0], M[r - 1, 0]
        new_upw, new_up0 = upw, up0
        if f0 != -1 and upw != -1:
            if f0 >= 0 and upw == -2 and close(upw_m, f0):
                new_upw = f0
            if up0 != -1 and f0 >= 0 and up0 == -2 and close(um0, f0):
                new_up0 = f0
        if w == 1:
            new_upw = new_up0
        S[r - 1, w - 1] = new_upw
        S[r - 1, 0] = new_up0
        S[r] = F
    return S.astype(np.int8)


def _inputs(h, w, seed, dense_mask=True):
    """8 sensors of refinement states: planar rectangles of up to 6 models inside a non-planar (-2) field with
    holes (-1), and closeness masks that let labels run far through the non-planar field."""
    rng = np.random.default_rng(seed)
    S = np.full((8, h, w), -2, np.int8)
    M = np.zeros((8, h, w), np.uint64)
    for s in range(8):
        nm = int(rng.integers(1, 7))
        for m in range(nm):
            r0, c0 = int(rng.integers(0, h)), int(rng.integers(0, w))
            S[s, r0:r0 + int(rng.integers(1, max(2, h // 3))), c0:c0 + int(rng.integers(1, max(2, w // 3)))] = m
        holes = rng.random((h, w)) < 0.04
        S[s][holes] = -1
        for _ in range(3):   # hole rectangles cut the chains
            r0, c0 = int(rng.integers(0, h)), int(rng.integers(0, w))
            S[s, r0:r0 + int(rng.integers(1, 4)), c0:c0 + int(rng.integers(1, w // 2 + 2))] = -1
        p = 0.9 if dense_mask else 0.5
        for m in range(nm):
            bit = (rng.random((h, w)) < p).astype(np.uint64) << np.uint64(m)
            M[s] |= bit
    return S, M


@pytest.mark.parametrize("seed,dense", [(1, True), (2, False), (3, True)])
def test_banded_sweeps_equal_python_restatement(seed, dense):
    h, w = 37, 70
    S, M = _inputs(h, w, seed, dense)
    ref = np.stack([_refine_ref(S[s], M[s]) for s in range(8)])
    assert not np.array_equal(ref, S)            # the sweeps changed something
    for rb in (-1, -2, 0, 1, 3, 8, 16, 37):
        out = R.refine_eval(S, M, rb)
        assert np.array_equal(out, ref), (rb, np.argwhere(out != ref)[:5])


@pytest.mark.parametrize("h,w", [(240, 320), (480, 640), (120, 160), (65, 97), (200, 333), (512, 640)])
def test_banded_sweeps_equal_single_wave(h, w):
    for seed in (11, 12):
        S, M = _inputs(h, w, seed)
        one = R.refine_eval(S, M, 0)
        for rb in [r for r in (-1, -2, 4, 16, 32) if r < 0 or -(-h // r) <= 64]:
            assert np.array_equal(R.refine_eval(S, M, rb), one), (h, w, rb, seed)


def _no_wrap(S):
    """The same states with the last column unlabelled (-1): the second sweep's flat-index wrap push (column 0
    of row r+1 into (r, w-1)) can then never fire, so the wavefront needs no fallback."""
    S = S.copy()
    S[:, :, -1] = -1
    return S


@pytest.mark.parametrize("h,w", [(37, 70), (130, 203), (240, 320), (480, 640)])
def test_wavefront_sweeps_both_paths(h, w):
    """The wavefront sweeps (the default refinement path) on both of its paths: no wrap push (pure wavefront,
    checked against the sequential restatement / single-wave kernel) and wrap pushes firing (the fallback
    sensor(s) redo the second sweep)."""
    seen_fb = 0
    for seed in (21, 22, 23):
        S, M = _inputs(h, w, seed)
        for St, want_fb in ((_no_wrap(S), False), (S, None)):
            ref = (np.stack([_refine_ref(St[s], M[s]) for s in range(8)]) if h * w <= 37 * 70
                   else R.refine_eval(St, M, 0))
            for rb in (-1, -2):   # LDS-pipelined bands (default) and barrier per diagonal
                out, nfb = R.refine_eval(St, M, rb, return_fallbacks=True)
                assert np.array_equal(out, ref), (h, w, seed, rb, np.argwhere(out != ref)[:5])
                if want_fb is False:
                    assert nfb == 0
                else:
                    seen_fb += nfb
    assert seen_fb > 0   # the random fields do make the wrap push fire somewhere


@pytest.mark.parametrize("h,w", [(37, 70), (240, 320)])
def test_wavefront_sweeps_wide_labels(h, w):
    """Labels and closeness bits above 30 (sensors with more than 30 models): the pipelined sweeps take their
    64-bit mask path there, checked like the narrow one."""
    for seed in (31, 32):
        S, M = _inputs(h, w, seed)
        S = np.where(S >= 0, S + 40, S).astype(np.int8)
        M = M << np.uint64(40)
        S[3] = np.where(S[3] >= 0, S[3] - 40, S[3])   # one narrow sensor beside the wide ones
        M[3] = M[3] >> np.uint64(40)
        ref = (np.stack([_refine_ref(S[s], M[s]) for s in range(8)]) if h * w <= 37 * 70
               else R.refine_eval(S, M, 0))
        for rb in (-1, -2):
            out = R.refine_eval(S, M, rb)
            assert np.array_equal(out, ref), (h, w, seed, rb, np.argwhere(out != ref)[:5])
