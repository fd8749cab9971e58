"""Fused FFN activation dropout(relu(h)) (models/modules/ffn.py, csrc/ffn_glue.hip): the reference's
``self.dropout2(self.activation(self.linear1(src)))`` (unimodal_deformable_transformer.py:233-236,
360-362).

CPU / fp32 / eval: exactly ``dropout(relu(h))``.  GPU bf16: relu bit-exact without dropout; with
dropout p the kept fraction of the positive elements is 1 - p and out / dx equal the ATen math run
with the kernel's own mask (recovered from the output: out > 0 exactly where h > 0 and kept)."""
import pytest
import torch
import torch.nn.functional as F

from conftest import PKG

FF = PKG.models.modules.ffn


def test_cpu_is_plain_dropout_relu():
    torch.manual_seed(0)
    drop = torch.nn.Dropout(0.1).eval()
    h = torch.randn(4, 64, 2048)
    torch.testing.assert_close(FF.relu_dropout(h, F.relu, drop), F.relu(h), rtol=0, atol=0)


@pytest.mark.gpu
def test_relu_only_bit_exact(dev):
    torch.manual_seed(1)
    drop = torch.nn.Dropout(0.1).eval()
    h = torch.randn(8, 1920, 2048, device=dev).bfloat16().requires_grad_(True)
    out = FF.relu_dropout(h, F.relu, drop)
    dy = torch.randn_like(out)
    out.backward(dy)
    h2 = h.detach().clone().requires_grad_(True)
    ref = F.relu(h2)
    ref.backward(dy)
    torch.testing.assert_close(out, ref, rtol=0, atol=0)
    torch.testing.assert_close(h.grad, h2.grad, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [8, 4096 * 2048, 100 * 8 * 2048])
def test_dropout_relu_matches_aten_math_with_its_mask(dev, n):
    torch.manual_seed(n)
    p = 0.1
    drop = torch.nn.Dropout(p).train()
    h = torch.randn(n, device=dev).bfloat16().requires_grad_(True)
    out = FF.relu_dropout(h, F.relu, drop)
    dy = torch.randn(n, device=dev).bfloat16()
    out.backward(dy)
    pos = h.detach() > 0
    keep = out.detach() > 0
    assert not bool((keep & ~pos).any())
    if n > 1000:
        rate = (keep.sum() / pos.sum()).item()
        assert abs(rate - (1 - p)) < 0.005, rate
    scale = 1.0 / (1.0 - p)
    ref = (F.relu(h.detach().float()) * keep * scale).bfloat16()
    torch.testing.assert_close(out.detach(), ref, rtol=2 ** -8, atol=0)
    rdx = (dy.float() * keep * scale).bfloat16()
    torch.testing.assert_close(h.grad, rdx, rtol=2 ** -8, atol=0)
    assert bool((h.grad[~keep] == 0).all())


@pytest.mark.gpu
def test_fresh_mask_per_call(dev):
    drop = torch.nn.Dropout(0.1).train()
    h = torch.ones(1 << 20, device=dev).bfloat16()
    a = FF.relu_dropout(h, F.relu, drop)
    b = FF.relu_dropout(h, F.relu, drop)
    assert (a != b).float().mean().item() > 0.1


@pytest.mark.gpu
@pytest.mark.parametrize("train", [False, True])
def test_nan_propagates_as_aten(dev, train):
    """ATen's relu keeps NaN (and x * mask keeps it through dropout): a diverging FFN shows up as
    NaN instead of being zeroed by the fused kernel."""
    drop = torch.nn.Dropout(0.5).train(train)
    h = torch.randn(4096, device=dev)
    h[::7] = float("nan")
    h = h.bfloat16()
    out = FF.relu_dropout(h, F.relu, drop)
    assert bool(torch.isnan(out[::7]).all())
    assert not bool(torch.isnan(out[1::7]).any())


@pytest.mark.gpu
def test_graph_replays_draw_fresh_masks(dev):
    """The dropout seed is drawn on the device inside the captured region, so every replay of a
    graph draws new keep bits (a seed frozen at capture would reuse one mask for every step):
    the FFN relu_dropout and the fused add + LayerNorm's residual dropout, replayed twice."""
    AN = PKG.models.modules.add_norm
    torch.manual_seed(3)
    drop = torch.nn.Dropout(0.1).train()
    norm = torch.nn.LayerNorm(512).to(dev)
    h = torch.randn(256, 2048, device=dev).abs().bfloat16() + 0.5  # relu keeps every element
    r = torch.randn(256, 512, device=dev)
    y = torch.randn(256, 512, device=dev).bfloat16()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side), torch.autocast("cuda", dtype=torch.bfloat16):
        FF.relu_dropout(h, F.relu, drop)
        AN.add_layer_norm(r, y, norm, drop)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g), torch.autocast("cuda", dtype=torch.bfloat16):
        out_f = FF.relu_dropout(h, F.relu, drop)
        out_n = AN.add_layer_norm(r, y, norm, drop)
    masks, norms = [], []
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        masks.append(out_f != 0)
        norms.append(out_n.clone())
    for m in masks:
        assert abs(m.float().mean().item() - 0.9) < 0.01
    assert (masks[0] != masks[1]).float().mean().item() > 0.1  # independent masks differ in ~18 %
    assert not torch.equal(norms[0], norms[1])


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols", [(15360, 2048), (16120, 2048), (800, 2048), (1001, 1032), (37, 1024)])
def test_backward_hands_over_column_sums(dev, rows, cols):
    """The backward writes dx and its column sums in one pass (mfl_relu_dropout_backward_colsum) and
    hands them to the Linear that produced h (linear1's bias gradient, linear._given_colsum): dx equal
    to the plain kernel's, the sums equal to dx's fp64 column sums to fp32 rounding; the Linear's bias
    gradient through them equals the one from its own column-sum pass."""
    torch.manual_seed(5)
    drop = torch.nn.Dropout(0.1).train()
    lin = PKG.models.modules.linear.Linear(256, cols).to(dev)
    x = torch.randn(rows, 256, device=dev)
    dy = torch.randn(rows, cols, device=dev).bfloat16()
    seed = torch.randint(0, 2 ** 62, (1,), device=dev, dtype=torch.int64)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        h = lin(x)
    out = FF._ReluDropout.apply(h, 0.1, seed)
    out.backward(dy)
    g1 = lin.bias.grad.clone()
    dx = torch.empty_like(out)
    lib = PKG._native.load_library()
    assert lib.mfl_relu_dropout_backward(dy.data_ptr(), out.data_ptr(), out.numel(), 0.1, 1, dx.data_ptr(),
                                         PKG._native.stream_handle(dev)) == 0
    want = dx.double().sum(0)
    torch.testing.assert_close(g1.double(), want, rtol=1e-5, atol=1e-5 * want.abs().max().item())
    lin.bias.grad = None
    PKG.models.modules.linear._AutocastLinear.backward  # (the consumer: _given_colsum)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        h2 = lin(x)
    h2.backward(dx)  # no handed-over sums: the Linear's own column-sum pass
    torch.testing.assert_close(lin.bias.grad.double(), want, rtol=1e-5, atol=1e-5 * want.abs().max().item())
