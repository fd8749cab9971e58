"""Fused MSDA prologue (msda_hip_prologue_forward / _backward through the C-ABI) against the
reference's own PyTorch composition of the same step (models/modules/attention.py:468-483:
softmax over L*P, loc = ref + off / T_l or the box form ref0 + off / P * ref1 * 0.5), in
fp64 / fp32 and under bf16 autocast, forward and backward.

Tolerances: fp64 1e-12; fp32 locations bitwise (same two operations), softmax and its
gradient 1e-6; bf16 autocast: locations bitwise (the kernel rounds off / T_l to bf16 exactly
where PyTorch's promotion does), gradients within one bf16 ulp."""
import pytest
import torch
import torch.nn.functional as F

from conftest import PKG

pytestmark = pytest.mark.gpu
msda = PKG.msda


def reference_prologue(off, logits, ref, shapes):
    """attention.py:468-483 restated (the module's composite path)."""
    B, Lq, M, L, P = off.shape
    aw = F.softmax(logits, -1).view(B, Lq, M, L, P)
    if ref.shape[-1] == 1:
        normalizer = torch.tensor(shapes, device=off.device)
        loc = ref[:, :, None, :, None, 0] + off / normalizer[None, None, None, :, None]
    else:
        loc = ref[:, :, None, :, None, 0] + off / P * ref[:, :, None, :, None, 1] * 0.5
    return loc, aw


def make(B, Lq, M, L, P, ref_dim, dtype, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    off = (torch.randn(B, Lq, M, L, P, generator=g, dtype=torch.float64) * 3).to(dev, dtype)
    logits = torch.randn(B, Lq, M, L * P, generator=g, dtype=torch.float64).to(dev, dtype)
    cd = torch.float64 if dtype == torch.float64 else torch.float32
    ref = torch.rand(B, Lq, L, ref_dim, generator=g, dtype=torch.float64).to(dev, cd)
    gl = torch.randn(B, Lq, M, L, P, generator=g, dtype=torch.float64).to(dev, cd)
    ga = torch.randn(B, Lq, M, L, P, generator=g, dtype=torch.float64).to(dev, cd)
    return off, logits, ref, gl, ga


def run_both(off, logits, ref, gl, ga, shapes):
    outs = []
    for fused in (True, False):
        o = off.detach().clone().requires_grad_(True)
        lg = logits.detach().clone().requires_grad_(True)
        r = ref.detach().clone().requires_grad_(True)
        if fused:
            loc, aw = msda.msda_prologue_apply(o, lg, r, shapes)
        else:
            loc, aw = reference_prologue(o, lg, r, shapes)
        (loc * gl).sum().backward(retain_graph=True)
        (aw * ga).sum().backward()
        outs.append((loc.detach(), aw.detach(), o.grad, lg.grad, r.grad))
    return outs


@pytest.mark.parametrize("ref_dim", [1, 2])
@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-12), (torch.float32, 1e-6)])
@pytest.mark.parametrize("B,Lq,M,L,P,shapes", [(2, 37, 8, 4, 4, [1024, 512, 256, 128]),  # per-sample kernels
                                              (1, 9, 4, 2, 8, [300, 150]),
                                              (1, 5, 2, 3, 2, [17, 9, 5]),                 # generic kernels
                                              (3, 11, 16, 1, 4, [64]), (2, 7, 3, 4, 4, [40, 20, 10, 5]),
                                              (8, 1030, 8, 4, 4, [1024, 512, 256, 128]),   # item-per-thread path
                                              (4, 2050, 8, 2, 8, [300, 150])])
def test_matches_reference_composition(dev, ref_dim, dtype, tol, B, Lq, M, L, P, shapes):
    off, logits, ref, gl, ga = make(B, Lq, M, L, P, ref_dim, dtype, dev)
    (loc, aw, go, glg, gr), (loc_r, aw_r, go_r, glg_r, gr_r) = run_both(off, logits, ref, gl, ga, shapes)
    assert loc.dtype == loc_r.dtype and aw.dtype == aw_r.dtype
    if dtype == torch.float32:
        assert torch.equal(loc, loc_r)
    torch.testing.assert_close(loc, loc_r, rtol=tol, atol=tol)
    torch.testing.assert_close(aw, aw_r, rtol=tol, atol=tol)
    torch.testing.assert_close(go, go_r, rtol=tol, atol=tol)
    torch.testing.assert_close(glg, glg_r, rtol=tol, atol=tol)
    torch.testing.assert_close(gr, gr_r, rtol=tol * 10, atol=tol * 10)


@pytest.mark.parametrize("ref_dim", [1, 2])
@pytest.mark.parametrize("L,P", [(4, 4), (3, 2)])
@pytest.mark.parametrize("Lq", [64, 1200])  # per-sample / item-per-thread kernels
def test_bf16_autocast_promotion(dev, ref_dim, L, P, Lq):
    """Under autocast the projections emit bf16: off / T_l is a bf16 tensor, the softmax runs in
    fp32 and the sum with the fp32 reference is fp32 (the module's composite path)."""
    B, M = 8, 8
    shapes = [1024, 512, 256, 128][:L]
    off, logits, ref, gl, ga = make(B, Lq, M, L, P, ref_dim, torch.bfloat16, dev, seed=1)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        (loc, aw, go, glg, gr), (loc_r, aw_r, go_r, glg_r, gr_r) = run_both(off, logits, ref, gl, ga, shapes)
    assert loc.dtype == torch.float32 and aw.dtype == torch.float32
    assert go.dtype == torch.bfloat16 and glg.dtype == torch.bfloat16
    assert torch.equal(loc, loc_r)
    torch.testing.assert_close(aw, aw_r, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(go.float(), go_r.float(), rtol=8e-3, atol=1e-6)
    torch.testing.assert_close(glg.float(), glg_r.float(), rtol=8e-3, atol=1e-6)
    torch.testing.assert_close(gr, gr_r, rtol=1e-5, atol=1e-5)


def test_module_uses_fused_prologue_and_matches_composite(dev):
    """MSDeformAttn on the GPU takes the fused path; the CPU composite (reference math) gives
    the same output and gradients in fp64."""
    torch.manual_seed(0)
    attn = PKG.models.modules.attention.MSDeformAttn(64, 4, 8, 4).double()
    shapes = [32, 16, 8, 4]
    S = sum(shapes)
    q = torch.randn(2, 20, 64, dtype=torch.float64)
    ref = torch.rand(2, 20, 4, 1, dtype=torch.float64)
    x = torch.randn(2, S, 64, dtype=torch.float64)
    st = torch.tensor(shapes)
    lsi = torch.tensor([0, 32, 48, 56])
    from oracle.cpu_model import oracle_core
    outs = []
    for device in ("cpu", dev):
        a = attn.to(device)
        qq, rr, xx = (t.detach().to(device).requires_grad_(True) for t in (q, ref, x))
        if device == "cpu":
            with oracle_core(PKG):
                y = a(qq, rr, xx, st, lsi)
        else:
            y = a(qq, rr, xx, st.to(device), lsi.to(device))
        y.square().sum().backward()
        outs.append([t.detach().cpu() for t in (y, qq.grad, rr.grad, xx.grad)])
        a.zero_grad()
    for u, v in zip(*outs):
        torch.testing.assert_close(u, v, rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("Lq,ref_dim", [(1920, 1), (100, 2), (37, 1)])
def test_query_prologue_matches_two_projection_form(dev, Lq, ref_dim):
    """_QueryPrologue (both query projections as one GEMM into [offsets | logits] rows, the strided
    prologue kernels reading / writing those rows; msda_hip_prologue_*_ex) against the
    two-projection form (linear_pair + the prologue on separate tensors), bf16 autocast with the
    trainer's shadow layout (the two weights back to back): locations, weights and every
    gradient agree to bf16 rounding of the projections."""
    from torch import nn
    att = PKG.models.modules.attention
    torch.manual_seed(3)
    m = att.MSDeformAttn(256, 4, 8, 4).to(dev)
    nn.init.normal_(m.sampling_offsets.weight, std=0.02)
    B, L, M, P = 2, 4, 8, 4
    shapes = [64, 32, 16, 8]
    x = torch.randn(B, Lq, 256, device=dev).requires_grad_(True)
    ref = torch.rand(B, Lq, L, ref_dim, device=dev).requires_grad_(True)
    a, b = m.sampling_offsets, m.attention_weights
    wc = torch.cat((a.weight, b.weight)).to(torch.bfloat16)
    bc = torch.cat((a.bias, b.bias)).to(torch.bfloat16)
    wca, wcb, bca, bcb = wc[:128], wc[128:], bc[:128], bc[128:]  # adjacent views, as the trainer's shadow
    gl = torch.randn(B, Lq, M, L, P, device=dev)
    ga = torch.randn(B, Lq, M, L, P, device=dev)

    def grads(loc, aw):
        params = [x, ref, a.weight, a.bias, b.weight, b.bias]
        return torch.autograd.grad((loc * gl).sum() + (aw * ga).sum(), params)

    PKG._trace.clear()
    loc1, aw1 = att._QueryPrologue.apply(x.to(torch.bfloat16), a.weight, a.bias, b.weight, b.bias, wca, bca, wcb, bcb,
                                         ref, tuple(shapes), (B, Lq, M, L, P))
    assert PKG._trace.hits.get("query_prologue") == 1
    g1 = grads(loc1, aw1)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        for mod, w, bb in ((a, wca, bca), (b, wcb, bcb)):
            mod.set_bf16_shadow(w, bb)
        off, lg = PKG.models.modules.linear.linear_pair(x, a, b)
    loc2, aw2 = msda.msda_prologue_apply(off.view(B, Lq, M, L, P), lg.view(B, Lq, M, L * P), ref, shapes)
    g2 = grads(loc2, aw2)
    torch.testing.assert_close(aw1, aw2, rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(loc1, loc2, rtol=2e-2, atol=2e-3)
    for n, u, v in zip(("x", "ref", "w_off", "b_off", "w_aw", "b_aw"), g1, g2):
        err = (u.float() - v.float()).norm() / v.float().norm().clamp_min(1e-12)
        assert err < 2e-2, (n, err.item())


@pytest.mark.parametrize("ref_dim", [1, 2])
@pytest.mark.parametrize("B,Lq,M,L,P", [(8, 1920, 8, 4, 4), (2, 77, 4, 2, 8), (3, 45, 8, 1, 16)])
def test_level_major_rows_equal_reference_layout(dev, ref_dim, B, Lq, M, L, P):
    """The level-major prologue (msda_hip_prologue_*_layout with MSDA_COORD_LEVEL_MAJOR: loc / aw
    (B, M, L, Lq, P), one workgroup per 32 queries x all heads) against the reference-layout
    kernels on one [offsets | logits] row buffer: locations, weights and the offsets / logits
    gradients bit for bit; the reference-point gradient sums the heads in another order (fp32
    rounding only)."""
    shapes = [1024, 512, 256, 128][:L] if L <= 4 else [64] * L
    n = M * L * P
    g = torch.Generator().manual_seed(3)
    y = (torch.randn(B * Lq, 2 * n, generator=g) * 2).to(dev, torch.bfloat16)
    ref = torch.rand(B, Lq, L, ref_dim, generator=g).to(dev)
    gl = torch.randn(B, Lq, M, L, P, generator=g).to(dev)
    ga = torch.randn(B, Lq, M, L, P, generator=g).to(dev)
    loc, aw = msda.prologue_forward_rows(y, B, Lq, M, L, P, ref, shapes)
    loc_m, aw_m = msda.prologue_forward_rows(y, B, Lq, M, L, P, ref, shapes, layout=msda.LEVEL_MAJOR)
    assert tuple(loc_m.shape) == (B, M, L, Lq, P)
    assert torch.equal(loc, loc_m.permute(0, 3, 1, 2, 4))
    g2, gr = msda.prologue_backward_rows(gl, ga, aw, y, ref, shapes)
    lmj = lambda t: t.permute(0, 2, 3, 1, 4).contiguous()  # noqa: E731
    g2m, grm = msda.prologue_backward_rows(lmj(gl), lmj(ga), aw_m, y, ref, shapes, layout=msda.LEVEL_MAJOR)
    if B * Lq * M >= 65536:  # the reference layout's item-per-thread kernels: the same sums in the same order
        assert torch.equal(aw, aw_m.permute(0, 3, 1, 2, 4)) and torch.equal(g2, g2m)
    else:  # (small calls take its per-sample kernels: softmax sums reduced in another order)
        torch.testing.assert_close(aw_m.permute(0, 3, 1, 2, 4), aw, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(g2m.float(), g2.float(), rtol=8e-3, atol=1e-6)
    torch.testing.assert_close(grm, gr, rtol=1e-5, atol=1e-6)


def test_module_level_major_path_matches_reference_layout(dev, monkeypatch):
    """MSDeformAttn at the bench's encoder call under bf16 autocast (B=8, T=1024 pyramid, 8 heads):
    the fused path keeps the coordinates level-major between the prologue, the MSDA kernels and
    their backward; against the same module with the reference layout throughout
    (MSDA_HIP_LEVEL_MAJOR=0): the output bit for bit, every gradient to fp32 rounding of the
    reference-point sums."""
    torch.manual_seed(1)
    attn = PKG.models.modules.attention.MSDeformAttn(512, 4, 8, 4).to(dev)
    shapes = [1024, 512, 256, 128]
    S = sum(shapes)
    g = torch.Generator().manual_seed(2)
    q = torch.randn(8, S, 512, generator=g).to(dev)
    x = torch.randn(8, S, 512, generator=g).to(dev)
    ref = torch.cat([(torch.arange(t) + 0.5) / t for t in shapes]).view(1, S, 1, 1).expand(8, S, 4, 1).to(dev)
    gout = torch.randn(8, S, 512, generator=g).to(dev)
    st, lsi = torch.tensor(shapes, device=dev), torch.tensor([0, 1024, 1536, 1792], device=dev)
    runs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("MSDA_HIP_LEVEL_MAJOR", flag)
        attn.zero_grad()
        qq, xx = q.clone().requires_grad_(True), x.clone().requires_grad_(True)
        PKG._trace.clear()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = attn(qq, ref, xx, st, lsi)
        y.float().backward(gout)
        torch.cuda.synchronize()
        assert (PKG._trace.hits.get("msda_level_major", 0) > 0) == (flag == "1")
        runs.append((y.detach(), qq.grad, xx.grad) + tuple(p.grad.clone() for p in attn.parameters()))
    assert torch.equal(runs[0][0], runs[1][0])
    for a, b in zip(runs[0][1:], runs[1][1:]):
        torch.testing.assert_close(a, b, rtol=2e-3, atol=1e-5)
