"""include/host_lsa.h: the DVC step's host matching in one native call, against scipy's
linear_sum_assignment (the reference matcher's solver, models/matcher.py:86-94) on the same matrices —
including integer-valued costs full of ties, where the assignment depends on the algorithm's scan
order and tie rule — and against the Python host step it replaces (HungarianMatcher.solve_levels +
get_src_permutation_idx)."""
import ctypes

import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment

from conftest import PKG


def _lsa(cost):
    lib = PKG._native.load_library()
    c = np.ascontiguousarray(cost, dtype=np.float64)
    k = min(c.shape)
    rows, cols = np.zeros(k, np.int64), np.zeros(k, np.int64)
    rc = lib.mfl_lsa(c.ctypes.data, c.shape[0], c.shape[1], rows.ctypes.data, cols.ctypes.data)
    return rc, rows, cols


@pytest.mark.parametrize("kind", ["float", "int", "const"])
def test_lsa_matches_scipy(kind):
    rng = np.random.default_rng(3)
    for trial in range(400):
        nr, nc = int(rng.integers(1, 13)), int(rng.integers(1, 13))
        if kind == "float":
            c = rng.standard_normal((nr, nc))
        elif kind == "int":
            c = rng.integers(0, 4, (nr, nc)).astype(np.float64)
        else:
            c = np.full((nr, nc), 2.5)
        rc, r, k = _lsa(c)
        assert rc == 0
        want_r, want_c = linear_sum_assignment(c)
        assert np.array_equal(r, want_r) and np.array_equal(k, want_c), (trial, c, r, k, want_r, want_c)


def test_lsa_infeasible_and_invalid():
    c = np.array([[np.inf, 1.0], [np.inf, 2.0]])
    assert _lsa(c)[0] == 3  # scipy raises "cost matrix is infeasible"
    with pytest.raises(ValueError):
        linear_sum_assignment(c)
    c = np.array([[np.nan, 1.0], [0.0, 2.0]])
    assert _lsa(c)[0] == 2


def test_lsa_levels_matches_python_host_step():
    """mfl_lsa_levels on a request buffer of the staged DVC loss equals solve_levels' per-clip scipy
    calls and the Python index building of StagedDVCLoss.host (bench shape: 6 levels, 8 clips, 100
    predictions, 1-7 targets a clip; float64 costs with ties, as the request is)."""
    rng = np.random.default_rng(11)
    L, B, Q = 6, 8, 100
    counts = rng.integers(1, 8, B)
    bounds = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    n_tgt = int(bounds[-1])
    cost = rng.standard_normal((L, B, Q, n_tgt))
    cost[..., : n_tgt // 3] = np.round(cost[..., : n_tgt // 3])  # ties
    lib = PKG._native.load_library()
    src, tgt = np.zeros((L, n_tgt), np.int64), np.zeros((L, n_tgt), np.int64)
    idx = np.zeros((L, 2, n_tgt), np.int64)
    rc = lib.mfl_lsa_levels(cost.ctypes.data, L, B, Q, n_tgt, bounds.ctypes.data, src.ctypes.data, tgt.ctypes.data,
                            idx.ctypes.data)
    assert rc == 0
    for lvl in range(L):
        for b in range(B):
            i, j = linear_sum_assignment(cost[lvl, b, :, bounds[b]:bounds[b + 1]])
            s = slice(bounds[b], bounds[b + 1])
            assert np.array_equal(src[lvl, s], i) and np.array_equal(tgt[lvl, s], j)
            assert np.array_equal(idx[lvl, 0, s], np.full(len(i), b))
            assert np.array_equal(idx[lvl, 1, s], i[np.argsort(j, kind="stable")])
    # bad arguments: bounds not covering n_tgt, more targets than predictions
    assert lib.mfl_lsa_levels(cost.ctypes.data, L, B, Q, n_tgt + 1, bounds.ctypes.data, src.ctypes.data,
                              tgt.ctypes.data, idx.ctypes.data) == 1
    small = np.ascontiguousarray(cost[:, :, :1])
    assert lib.mfl_lsa_levels(small.ctypes.data, L, B, 1, n_tgt, bounds.ctypes.data, src.ctypes.data,
                              tgt.ctypes.data, idx.ctypes.data) == 1


def test_solve_levels_native_matches_scipy_path(monkeypatch):
    """HungarianMatcher.solve_levels through the native call returns the scipy path's index tensors."""
    HM = PKG.models.matcher.HungarianMatcher
    rng = np.random.default_rng(5)
    B, Q = 4, 30
    sizes = [3, 1, 5, 2]
    n_tgt = sum(sizes)
    shapes = [(B, Q)] * 3
    h = np.concatenate([rng.random(3 * B * Q * n_tgt), np.ones(2)])  # (float64, as level_costs' request)
    meta = (shapes, sizes, n_tgt, 2)
    monkeypatch.setenv("MFL_HOST_LSA", "0")
    want = HM.solve_levels(torch.from_numpy(h), meta)
    monkeypatch.setenv("MFL_HOST_LSA", "1")
    got = HM.solve_levels(torch.from_numpy(h), meta)
    assert len(got) == len(want)
    for lg, lw in zip(got, want):
        for (gi, gj), (wi, wj) in zip(lg, lw):
            assert torch.equal(gi, wi) and torch.equal(gj, wj) and gi.dtype == torch.int64


def test_level_costs_all_levels_at_once_equal_per_level():
    """HungarianMatcher.level_costs over several decoder levels builds every level's cost rows in one
    matrix: bit for bit the per-level costs (each computed alone) concatenated, and the same flags."""
    import torch
    from conftest import PKG
    g = torch.Generator().manual_seed(3)
    m = PKG.models.matcher.HungarianMatcher(cost_class=1, cost_segment=5, cost_giou=2)
    B, Q, L = 3, 7, 4
    outs = [{"pred_segments": torch.rand(B, Q, 2, generator=g)} for _ in range(L)]
    targets = [{"segments": torch.rand(n, 2, generator=g) * 0.5 + 0.1} for n in (2, 3, 1)]
    joint, meta = m.level_costs(outs, targets)
    parts = [m.level_costs([o], targets)[0] for o in outs]
    n = B * Q * sum(len(t["segments"]) for t in targets)
    assert torch.equal(joint[:L * n], torch.cat([p[:n] for p in parts]))
    assert torch.equal(joint[L * n:], torch.cat([p[n:n + 1] for p in parts] + [parts[0][n + 1:]]))
    assert meta[3] == L + 1 and meta[0] == [(B, Q)] * L
