"""The oracle pinned against golden vectors produced by the real reference (CPU).

tests/golden/make_golden.py ran models/modules/attention.py:331-383 (and the module /
transformer levels) of /root/reference on CPU; these tests check the numpy restatement
(oracle/msda_oracle.py) and the grid_sample restatement (oracle/msda_grid_sample.py)
reproduce those outputs before anything is compared against them.
"""
import numpy as np
import pytest
import torch

from oracle import msda_oracle as O
from oracle.msda_grid_sample import msda_core_grid_sample


def _np(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("name,rtol,atol", [("op_border_f64", 1e-12, 1e-12), ("op_border_f32", 2e-5, 2e-6)])
def test_numpy_oracle_matches_reference(golden, name, rtol, atol):
    g = golden(name)
    shapes = g["shapes"].tolist()
    out = O.msda_forward(_np(g["value"]), shapes, _np(g["loc"]), _np(g["aw"]))
    np.testing.assert_allclose(out, _np(g["out"]), rtol=rtol, atol=atol)
    gv, gl, ga = O.msda_backward(_np(g["value"]), shapes, _np(g["loc"]), _np(g["aw"]), _np(g["grad_out"]))
    np.testing.assert_allclose(gv, _np(g["grad_value"]), rtol=rtol, atol=atol)
    np.testing.assert_allclose(ga, _np(g["grad_aw"]), rtol=rtol, atol=atol)
    # grad_loc carries T_l * sum_c(...): scale atol by the level length
    np.testing.assert_allclose(gl, _np(g["grad_loc"]), rtol=rtol, atol=atol * 64)


def test_numpy_oracle_border_gradient_zero_exactly_at_clamp(golden):
    g = golden("op_border_f64")
    gl = _np(g["grad_loc"])
    shapes = g["shapes"].tolist()
    loc = _np(g["loc"])
    for l, T in enumerate(shapes):
        y = (2 * loc[:, :, :, l] - 1 + 1) * (T / 2) - 0.5
        clamped = (y <= 0) | (y >= T - 1)
        assert clamped.any()
        assert np.all(gl[:, :, :, l][clamped] == 0.0)


def regenerate_enc_inputs(g):
    """Inputs of op_border_f32_enc.pt, regenerated from its seed exactly as make_golden.py drew them."""
    shapes = g["shapes"].tolist()
    B, M, D, Lq, P = (int(g[k]) for k in ("B", "M", "D", "Lq", "P"))
    gen = torch.Generator().manual_seed(int(g["seed"]))
    L, S = len(shapes), sum(shapes)
    value = torch.randn((B, S, M, D), generator=gen, dtype=torch.float64).float()
    loc = (torch.rand((B, Lq, M, L, P), generator=gen, dtype=torch.float64) * 1.4 - 0.2).float()
    for l, T in enumerate(shapes):
        pts = [0.5 / T, (T - 0.5) / T, 5.5 / T if T > 6 else 1.5 / T, 0.0, 1.0, -0.5, 1.5]
        flat = loc[:, 0, :, l].reshape(-1)
        for i, v in enumerate(pts):
            flat[i] = v
        loc[:, 0, :, l] = flat.view(loc[:, 0, :, l].shape)
    a = torch.rand((B, Lq, M, L, P), generator=gen, dtype=torch.float64) + 1e-5
    aw = (a / a.sum(-1, keepdim=True).sum(-2, keepdim=True)).float()
    gout = torch.randn((B, Lq, M * D), generator=gen, dtype=torch.float64).float()
    return shapes, value, loc, aw, gout


def test_numpy_oracle_enc_shape(golden):
    g = golden("op_border_f32_enc")
    shapes, value, loc, aw, gout = regenerate_enc_inputs(g)
    out = O.msda_forward(_np(value), shapes, _np(loc), _np(aw))
    np.testing.assert_allclose(out, _np(g["out"]), rtol=2e-5, atol=2e-6)
    gv, gl, ga = O.msda_backward(_np(value), shapes, _np(loc), _np(aw), _np(gout))
    np.testing.assert_allclose(ga, _np(g["grad_aw"]), rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(gl, _np(g["grad_loc"]), rtol=2e-4, atol=2e-4)
    np.testing.assert_allclose(gv.sum(-1), _np(g["grad_value_rowsum"]), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(gv[:, _np(g["grad_value_rows"])], _np(g["grad_value_at_rows"]), rtol=1e-4, atol=1e-6)


def test_grid_sample_restatement_matches_reference(golden):
    g = golden("op_border_f64")
    v, lc, a = (g[k].clone().requires_grad_(True) for k in ("value", "loc", "aw"))
    out = msda_core_grid_sample(v, g["shapes"].unsqueeze(-1), lc.unsqueeze(-1), a)
    out.backward(g["grad_out"])
    torch.testing.assert_close(out, g["out"], rtol=1e-13, atol=1e-13)
    torch.testing.assert_close(v.grad, g["grad_value"], rtol=1e-13, atol=1e-13)
    torch.testing.assert_close(lc.grad, g["grad_loc"], rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(a.grad, g["grad_aw"], rtol=1e-13, atol=1e-13)


def near_integer_locations(T, n=4096, seed=0):
    """fp32 locations one ulp either side of (k + 0.5) / T: their unnormalised y sits on or
    next to the integer k, where the operation order decides floor(y) (a plain
    loc*T - 0.5 picks the other segment for ~5% of them at T = 300 / 1000)."""
    rng = np.random.default_rng(seed)
    k = rng.integers(1, T - 2, size=n).astype(np.float64)
    loc = ((k + 0.5) / T).astype(np.float32)
    return np.nextafter(loc, np.where(rng.random(n) < 0.5, np.float32(-1), np.float32(2))).astype(np.float32)


@pytest.mark.parametrize("T", [1024, 1000, 300, 75, 50])
def test_fp32_coordinates_bit_identical_to_aten(T):
    """The tap segment of the fp32 oracle equals ATen's on locations where a one-ulp
    difference in y would move it.  The forward is continuous across segments, so the
    location gradient tells them apart: with v[k] = k*k the slope is 2k+1 on [k, k+1]
    and 2k-1 on [k-1, k]."""
    loc = near_integer_locations(T)
    value = (np.arange(T, dtype=np.float32) ** 2).reshape(1, T, 1, 1)
    loc5 = loc.reshape(1, -1, 1, 1, 1)
    aw5 = np.ones_like(loc5)
    ours = O.msda_forward(value, [T], loc5, aw5).reshape(-1)
    ref = msda_core_grid_sample(torch.from_numpy(value), [T], torch.from_numpy(loc5), torch.from_numpy(aw5))
    np.testing.assert_allclose(ours, ref.numpy().reshape(-1), rtol=2e-7)  # rounding only
    _, gl, _ = O.msda_backward(value, [T], loc5, aw5, np.ones((1, loc.size, 1), np.float32))
    lt = torch.from_numpy(loc5).clone().requires_grad_(True)
    msda_core_grid_sample(torch.from_numpy(value), [T], lt, torch.from_numpy(aw5)).sum().backward()
    np.testing.assert_allclose(gl.reshape(-1), lt.grad.numpy().reshape(-1), rtol=1e-6)


@pytest.mark.parametrize("padding", ["border", "zeros"])
def test_oracle_gradient_matches_finite_differences(padding):
    """fp64 central differences of the oracle forward reproduce its analytic backward
    (locations kept away from the kinks at integer / clamp positions)."""
    rng = np.random.default_rng(3)
    shapes = [9, 5, 3]
    B, M, D, Lq, P = 2, 2, 3, 4, 2
    S = sum(shapes)
    value = rng.standard_normal((B, S, M, D))
    loc = rng.uniform(-0.15, 1.15, size=(B, Lq, M, len(shapes), P))
    for l, T in enumerate(shapes):  # nudge off the kinks
        y = loc[:, :, :, l] * T - 0.5
        frac = y - np.floor(y)
        loc[:, :, :, l] += np.where(np.abs(frac) < 1e-3, 2e-3 / T, 0) + np.where(np.abs(frac - 1) < 1e-3, -2e-3 / T, 0)
    aw = rng.uniform(0.1, 1.0, size=loc.shape)
    gout = rng.standard_normal((B, Lq, M * D))
    gv, gl, ga = O.msda_backward(value, shapes, loc, aw, gout, padding=padding)
    f = lambda v, lc, a: float((O.msda_forward(v, shapes, lc, a, padding=padding) * gout).sum())  # noqa: E731
    eps = 1e-6
    for arr, grad in ((value, gv), (loc, gl), (aw, ga)):
        idxs = rng.choice(arr.size, size=12, replace=False)
        for i in idxs:
            saved = arr.flat[i]
            arr.flat[i] = saved + eps
            fp = f(value, loc, aw)
            arr.flat[i] = saved - eps
            fm = f(value, loc, aw)
            arr.flat[i] = saved
            np.testing.assert_allclose((fp - fm) / (2 * eps), grad.flat[i], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("padding", ["zeros", "border"])
def test_oracle_2d_form_matches_reference_ops_core(golden, padding):
    """ZEROS and the (L,2) / (...,2) extension form pinned: the reference's 2-D core
    (ops/functions/ms_deform_attn_func.py:44-71) on H = 1 maps, border as written and with the
    extension kernel's zero padding (tests/golden/make_golden.py::ops_api_case), incl. the y-gradient."""
    g = golden("ops_api_f64")
    shapes = [int(w) for _, w in g["shapes2d"].tolist()]
    r = g[padding]
    out, gv, gl, ga = O.msda_h1(_np(g["value"]), shapes, _np(g["loc2"]), _np(g["aw"]), _np(g["grad_out"]), padding)
    np.testing.assert_allclose(out, _np(r["out"]), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(gv, _np(r["grad_value"]), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(ga, _np(r["grad_aw"]), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(gl, _np(r["grad_loc"]), rtol=1e-11, atol=1e-10)
    if padding == "zeros":
        assert (_np(r["grad_loc"])[..., 1] != 0).any()  # the y-gradient is exercised
