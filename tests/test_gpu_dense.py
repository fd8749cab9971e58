"""Dense small-pyramid MSDA kernels (csrc/msda_win.hip dense_fwd_kernel / dense_bwd_kernel, round 6):
calls whose value pyramid has at most 128 rows per (b, m) — configs[2]'s video queries on the audio
pyramid (T_a = 50: S = 95, Lq = 1920) and the audio self-attention (S = Lq = 95) — against the oracle
restatement of the reference core (models/modules/attention.py:331-383, grid_sample bilinear,
align_corners=False) on the same bf16-rounded inputs in fp32, and against the row-block / gather
kernels they replace (MSDA_HIP_DENSE=0).

Tolerances as test_gpu_op.py's bf16 cases: outputs and grad_value within one bf16 rounding (2^-8
relative of the largest), grad_attn 1e-4, grad_loc 1e-4 relative + 2e-5 x T (the location scale)."""
import numpy as np
import pytest
import torch

from conftest import PKG
from oracle import msda_oracle as O
from test_gpu_op import _from_level_major, _np, _to_level_major, rand_case

pytestmark = pytest.mark.gpu
msda = PKG.msda


def cross_locations(B, Lq, M, shapes, P, seed, video=(1024, 512, 256, 128)):
    """Video tokens' sampling locations on the audio pyramid: each token's reference point (its
    position in the video pyramid) plus per-head offsets and a trained-like jitter."""
    g = torch.Generator().manual_seed(seed)
    L = len(shapes)
    ref = torch.cat([(torch.arange(t, dtype=torch.float32) + 0.5) / t for t in video])[:Lq]
    T = torch.tensor(shapes, dtype=torch.float32).view(1, 1, 1, L, 1)
    off = torch.randn(B, Lq, M, L, P, generator=g) * 1.5 / T
    return (ref.view(1, Lq, 1, 1, 1) + off).contiguous()


def run(value, shapes, loc, aw, gout, padding, layout):
    starts = O.level_starts(shapes)
    lm = layout == "level_major"
    v = value.cuda().requires_grad_(True)
    lc = (_to_level_major(loc) if lm else loc).cuda().requires_grad_(True)
    a = (_to_level_major(aw) if lm else aw).cuda().requires_grad_(True)
    out = msda.msda_apply(v, shapes, starts, lc, a, padding, layout=msda.LEVEL_MAJOR if lm else 0)
    out.backward(gout.cuda())
    torch.cuda.synchronize()
    gl, ga = (_from_level_major(t.grad) if lm else t.grad for t in (lc, a))
    return out.detach().cpu(), v.grad.cpu(), gl.cpu(), ga.cpu()


def check_oracle(value, shapes, loc, aw, gout, res, clips, padding):
    out, gv, gl, ga = res
    eps = 2 ** -8
    for b in clips:
        v32, g32 = value[b:b + 1].float(), gout[b:b + 1].float()
        r_out = O.msda_forward(_np(v32), shapes, _np(loc[b:b + 1]), _np(aw[b:b + 1]), padding=padding)
        r_gv, r_gl, r_ga = O.msda_backward(_np(v32), shapes, _np(loc[b:b + 1]), _np(aw[b:b + 1]), _np(g32),
                                            padding=padding)
        np.testing.assert_allclose(_np(out[b:b + 1]), r_out, rtol=eps, atol=eps * np.abs(r_out).max())
        np.testing.assert_allclose(_np(gv[b:b + 1]), r_gv, rtol=eps, atol=eps * np.abs(r_gv).max())
        np.testing.assert_allclose(_np(ga[b:b + 1]), r_ga, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(_np(gl[b:b + 1]), r_gl, rtol=1e-4, atol=2e-5 * max(shapes))


@pytest.mark.parametrize("layout", ["reference", "level_major"])
@pytest.mark.parametrize("padding", ["border", "zeros"])
def test_dense_cross_modal_call_matches_oracle(dev, monkeypatch, padding, layout):
    """configs[2]'s video -> audio call (multimodal_deformable_transformer.py:410-421): B clips, the
    T=1024 video pyramid's 1,920 tokens sampling the 95-row audio pyramid, as the bench runs it
    (level-major coordinates and the forward's tiles through msda_apply)."""
    monkeypatch.delenv("MSDA_HIP_DENSE", raising=False)
    shapes, B, M, D, P, Lq = [50, 25, 13, 7], 3, 8, 64, 4, 1920
    value, _, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=301, lo=0.0, hi=1.0)
    loc = cross_locations(B, Lq, M, shapes, P, seed=302)
    if layout == "level_major":
        assert msda.level_major_ok(value.cuda(), shapes, Lq, P)
    res = run(value, shapes, loc, aw, gout, padding, layout)
    check_oracle(value, shapes, loc, aw, gout, res, (0, B - 1), padding)


@pytest.mark.parametrize("shapes,P,Lq", [
    ([50, 25, 13, 7], 4, 95),      # configs[2]'s audio self-attention (S = Lq = 95)
    ([64, 32, 16, 8], 2, 200),     # 120 rows, P = 2
    ([128], 1, 77),                # one level at the 128-row limit, P = 1, a ragged last tile
    ([40, 20, 10], 4, 33),         # three levels, S = 70 (not a multiple of 16)
    ([3, 2, 1, 1], 4, 64),         # a pyramid of 7 rows: every tap near a border
])
@pytest.mark.parametrize("padding", ["border", "zeros"])
def test_dense_small_pyramids_match_oracle(dev, monkeypatch, shapes, P, Lq, padding):
    """Uniform locations in [-0.2, 1.2] (clamped / dropped taps at both borders), every clip."""
    monkeypatch.delenv("MSDA_HIP_DENSE", raising=False)
    B, M, D = 2, 8, 64
    value, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=311 + len(shapes) + P)
    res = run(value, shapes, loc, aw, gout, padding, "reference")
    check_oracle(value, shapes, loc, aw, gout, res, range(B), padding)


@pytest.mark.parametrize("layout", ["reference", "level_major"])
def test_dense_equals_replaced_kernels(dev, monkeypatch, layout):
    """The dense kernels against the gather forward / row-block backward they replace on the same
    inputs (MSDA_HIP_DENSE=0): the coordinate gradients come from the same dot products (bit for bit
    where both round the same fp32 dots), outputs and grad_value within one bf16 rounding."""
    shapes, B, M, D, P, Lq = [50, 25, 13, 7], 2, 8, 64, 4, 1920
    value, _, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=321, lo=0.0, hi=1.0)
    loc = cross_locations(B, Lq, M, shapes, P, seed=322)
    monkeypatch.delenv("MSDA_HIP_DENSE", raising=False)
    dense = run(value, shapes, loc, aw, gout, "border", layout)
    monkeypatch.setenv("MSDA_HIP_DENSE", "0")
    ref = run(value, shapes, loc, aw, gout, "border", layout)
    eps = 2 ** -8
    for x, y in zip(dense, ref):
        x, y = x.float(), y.float()
        torch.testing.assert_close(x, y, rtol=eps, atol=eps * y.abs().max().item())


def test_dense_backward_is_deterministic(dev, monkeypatch):
    """No atomics: two backward passes on the same inputs are bitwise equal."""
    monkeypatch.delenv("MSDA_HIP_DENSE", raising=False)
    shapes, B, M, D, P, Lq = [50, 25, 13, 7], 2, 8, 64, 4, 1920
    value, _, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.bfloat16, seed=331, lo=0.0, hi=1.0)
    loc = cross_locations(B, Lq, M, shapes, P, seed=332)
    r1 = run(value, shapes, loc, aw, gout, "border", "level_major")
    r2 = run(value, shapes, loc, aw, gout, "border", "level_major")
    for x, y in zip(r1, r2):
        assert torch.equal(x, y)
