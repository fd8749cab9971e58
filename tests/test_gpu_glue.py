"""Padding-row zeroing of MSDeformAttn's value (models/modules/attention.py::mask_padding_rows,
csrc/ffn_glue.hip ``mfl_zero_masked_rows``): the reference's
``value.masked_fill(input_padding_mask[..., None], 0)`` (attention.py:462-463) done in place on the
value projection's output, forward and backward, bit-exact against ATen's masked_fill."""
import pytest
import torch

from conftest import PKG

ATT = PKG.models.modules.attention


def test_cpu_is_masked_fill():
    v = torch.randn(2, 7, 16)
    m = torch.rand(2, 7) < 0.5
    torch.testing.assert_close(ATT.mask_padding_rows(v, m), v.masked_fill(m[..., None], 0.0), rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("kind", ["random", "none", "all", "tail"])
def test_zero_rows_matches_masked_fill(dev, dt, kind):
    torch.manual_seed(1)
    N, S, C = 3, 1920, 512
    if kind == "random":
        mask = torch.rand(N, S, device=dev) < 0.3
    elif kind == "none":
        mask = torch.zeros(N, S, dtype=torch.bool, device=dev)
    elif kind == "all":
        mask = torch.ones(N, S, dtype=torch.bool, device=dev)
    else:
        mask = torch.arange(S, device=dev)[None, :] >= torch.tensor([S, S // 2, 7], device=dev)[:, None]
    x = torch.randn(N, S, C, device=dev, dtype=dt, requires_grad=True)
    g = torch.randn(N, S, C, device=dev, dtype=dt)
    ref = x.detach().masked_fill(mask[..., None], 0.0)
    v = x * 1  # a fresh non-leaf tensor, as the value projection's output
    out = ATT.mask_padding_rows(v, mask)
    torch.testing.assert_close(out, ref, rtol=0, atol=0)
    out.backward(g)
    torch.testing.assert_close(x.grad, g.masked_fill(mask[..., None], 0.0), rtol=0, atol=0)


@pytest.mark.gpu
def test_module_with_padding_mask_uses_kernel(dev, monkeypatch):
    """MSDeformAttn with a padding mask goes through the in-place kernel and gives the
    masked_fill result (reference composition run with masked_fill for comparison)."""
    torch.manual_seed(2)
    attn = ATT.MSDeformAttn(64, 4, 4, 4).to(dev).double()
    shapes = [32, 16, 8, 4]
    S = sum(shapes)
    ts = torch.tensor(shapes, device=dev)
    lsi = torch.cat([ts.new_zeros(1), ts.cumsum(0)[:-1]])
    src = torch.randn(2, S, 64, device=dev, dtype=torch.float64)
    ref = torch.rand(2, S, 4, 1, device=dev, dtype=torch.float64)
    mask = torch.rand(2, S, device=dev) < 0.25
    calls = []
    real = ATT._ZeroPaddingRows.apply
    monkeypatch.setattr(ATT._ZeroPaddingRows, "apply", lambda *a: calls.append(1) or real(*a))
    out = attn(src, ref, src, ts, lsi, mask)
    assert calls
    monkeypatch.setattr(ATT, "mask_padding_rows", lambda v, m: v.masked_fill(m[..., None], 0.0))
    out2 = attn(src, ref, src, ts, lsi, mask)
    torch.testing.assert_close(out, out2, rtol=0, atol=0)
