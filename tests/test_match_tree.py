"""The SubgraphMatcher interpretation tree (A12, RegisterRGBD360.h:294; App. C.4) on the CPU: the product's
host search (r360_match_tree_search, no device) and the oracle's, both with forward checking, against an
exhaustive enumeration in pure Python on random match tables, including dense symmetric tables (many parallel
walls) where the old simple bound needed far more nodes; the node budget is reported, never silent.
MRPT's own matcher is absent here: the ordering (most matches, ties by matched reference area, first found)
is App. C.4's restatement — parity with MRPT unpinned."""
import numpy as np
import pytest

import rgbd360_amd as R
from oracle import oracle360 as O


def _tables(rng, ns, nt, p_unary, p_binary, symmetric):
    unary = rng.random((ns, nt)) < p_unary
    words = (ns * nt + 63) // 64
    ok = rng.random((ns, nt, ns, nt)) < p_binary
    if symmetric:
        ok = ok & ok.transpose(2, 3, 0, 1)
    binary = np.zeros((ns * nt, words), np.uint64)
    for i in range(ns):
        for j in range(nt):
            for k in range(ns):
                for l in range(nt):
                    if k != i and l != j and ok[i, j, k, l]:
                        bit = k * nt + l
                        binary[i * nt + j, bit // 64] |= np.uint64(1) << np.uint64(bit % 64)
    area = rng.uniform(0.2, 6.0, ns)
    return unary, binary, area, ok


def _exhaustive(unary, ok, area):
    """Every injective partial assignment consistent with the tables, in the tree's order (references in order,
    targets ascending, then unmatched); the first one with the most matches and, among those, the largest area."""
    ns, nt = unary.shape
    cur = [-1] * ns
    best = {"n": 0, "a": 0.0, "m": [-1] * ns}

    def rec(i, n, a):
        if i == ns:
            if n > best["n"] or (n == best["n"] and a > best["a"]):
                best.update(n=n, a=a, m=list(cur))
            return
        for t in range(nt):
            if not unary[i, t]:
                continue
            if all(cur[k] < 0 or (cur[k] != t and ok[i, t, k, cur[k]]) for k in range(i)):
                cur[i] = t
                rec(i + 1, n + 1, a + area[i])
                cur[i] = -1
        rec(i + 1, n, a)

    rec(0, 0, 0.0)
    return np.array(best["m"], np.int32)


@pytest.mark.parametrize("seed", range(12))
def test_tree_search_equals_exhaustive(seed):
    rng = np.random.default_rng(1000 + seed)
    ns, nt = int(rng.integers(1, 8)), int(rng.integers(1, 8))
    unary, binary, area, ok = _tables(rng, ns, nt, rng.uniform(0.3, 1.0), rng.uniform(0.3, 0.95), seed % 2 == 0)
    want = _exhaustive(unary, ok, area)
    got, nodes, trunc = R.match_tree_search(unary, binary, area)
    assert not trunc and (got == want).all(), (got, want)
    got_o, nodes_o, trunc_o = O.tree_search(unary, binary, area)
    assert not trunc_o and (got_o == want).all()
    assert nodes == nodes_o           # the same search in product and oracle


def test_dense_symmetric_tables_stay_exhaustive():
    """25 x 25 planes where most pairs are compatible (parallel walls; 90 % of the binary constraints hold): the
    forward-checking search finishes inside the default budget (1.3 M nodes) and both sides agree.  Random tables
    this dense with half the unary tests passing still exceed it: the search is NP-hard, and such a search is
    counted as truncated (test_budget_is_reported, r360_ctx_match_stats)."""
    rng = np.random.default_rng(7)
    unary, binary, area, _ = _tables(rng, 25, 25, 0.2, 0.9, True)
    got, nodes, trunc = R.match_tree_search(unary, binary, area)
    got_o, nodes_o, trunc_o = O.tree_search(unary, binary, area)
    assert not trunc and not trunc_o
    assert (got == got_o).all() and nodes == nodes_o
    assert (got >= 0).sum() >= 10


def test_budget_is_reported():
    rng = np.random.default_rng(3)
    unary, binary, area, _ = _tables(rng, 12, 12, 0.9, 0.9, True)
    _, nodes, trunc = R.match_tree_search(unary, binary, area, max_nodes=50)
    assert trunc and nodes == 51
    _, nodes_o, trunc_o = O.tree_search(unary, binary, area, max_nodes=50)
    assert trunc_o and nodes_o == 51
    _, _, trunc = R.match_tree_search(unary, binary, area)
    assert not trunc


def test_oracle_registration_reports_no_truncation():
    """The synthetic pair of every registration mode: the oracle's RegisterPbMap searches to the end."""
    rt = O.read_extrinsics(R.EXTRINSICS_DIR)
    seed = 360 << 16
    A = R.synth_path_pose(seed, 0)
    rel = np.eye(4, dtype=np.float32)
    rel[:3, 3] = [0, 0.25, 0.15]
    maps = []
    for P in (A, A @ rel):
        b, d = R.synth_frame_rt(240, 320, rt, seed, P)
        maps.append(O.PbMap(d.astype(np.float32) * np.float32(0.001), b, rt))
    for mode in range(4):
        r = O.register_pbmap(maps[0], maps[1], 25, mode)
        assert not r["truncated"] and r["nodes"] > 0
