"""Fused residual add + LayerNorm (models/modules/add_norm.py, csrc/add_layernorm.hip): the
reference's ``norm(x + dropout(y))`` of every deformable encoder / decoder layer
(unimodal_deformable_transformer.py:238-249, 362-373).

CPU: outside autocast / on the CPU it is exactly ``norm(r + y)``.
GPU: under bf16 autocast against an fp64 restatement of the same fp32 math (z = r + y with the
16-bit operand widened exactly, LayerNorm over the last dim) — outputs, both input gradients
(in their own dtypes) and gamma / beta gradients; fp32 tolerances, bf16 rounding for 16-bit
gradients."""
import pytest
import torch

from conftest import PKG

AN = PKG.models.modules.add_norm


def test_cpu_is_plain_layer_norm():
    torch.manual_seed(0)
    norm = torch.nn.LayerNorm(512)
    r, y = torch.randn(3, 7, 512), torch.randn(3, 7, 512)
    torch.testing.assert_close(AN.add_layer_norm(r, y, norm), norm(r + y), rtol=0, atol=0)


def _ref(r, y, w, b, eps, dout):
    r64 = r.detach().double().requires_grad_(True)
    y64 = y.detach().double().requires_grad_(True)
    w64 = w.detach().double().requires_grad_(True)
    b64 = b.detach().double().requires_grad_(True)
    out = torch.nn.functional.layer_norm(r64 + y64, (r.shape[-1],), w64, b64, eps)
    out.backward(dout.double())
    return out, r64.grad, y64.grad, w64.grad, b64.grad


@pytest.mark.gpu
@pytest.mark.parametrize("rows,d", [(15360, 512), (800, 512), (3, 256), (37, 1024)])
@pytest.mark.parametrize("rdt,ydt", [(torch.float32, torch.bfloat16), (torch.bfloat16, torch.bfloat16),
                                     (torch.float32, torch.float32)])
def test_fused_matches_fp64(dev, rows, d, rdt, ydt):
    torch.manual_seed(rows + d)
    norm = torch.nn.LayerNorm(d).to(dev)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.5, 0.5)
    r = (torch.randn(rows, d, device=dev) * 2 + 0.3).to(rdt).requires_grad_(True)
    y = torch.randn(rows, d, device=dev).to(ydt).requires_grad_(True)
    dout = torch.randn(rows, d, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = AN.add_layer_norm(r, y, norm)
    assert out.dtype == torch.float32
    out.backward(dout)
    assert r.grad.dtype == rdt and y.grad.dtype == ydt
    ro, rgr, rgy, rgw, rgb = _ref(r, y, norm.weight, norm.bias, norm.eps, dout)
    torch.testing.assert_close(out.double(), ro, rtol=1e-5, atol=1e-5)

    def close(a, ref, dt):
        tol = 2 ** -8 if dt == torch.bfloat16 else 1e-5
        torch.testing.assert_close(a.double(), ref, rtol=tol, atol=tol * ref.abs().max().item())
    close(r.grad, rgr, rdt)
    close(y.grad, rgy, ydt)
    close(norm.weight.grad, rgw, torch.float32)
    close(norm.bias.grad, rgb, torch.float32)


@pytest.mark.gpu
def test_unsupported_width_falls_back(dev):
    norm = torch.nn.LayerNorm(100).to(dev)
    r, y = torch.randn(4, 100, device=dev), torch.randn(4, 100, device=dev).bfloat16()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = AN.add_layer_norm(r, y, norm)
        ref = norm(r + y)
    torch.testing.assert_close(out, ref, rtol=0, atol=0)
