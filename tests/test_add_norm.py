"""Fused residual add + LayerNorm (models/modules/add_norm.py, csrc/add_layernorm.hip): the
reference's ``norm(x + dropout(y))`` of every deformable encoder / decoder layer
(unimodal_deformable_transformer.py:238-249, 362-373).

CPU: outside autocast / on the CPU it is exactly ``norm(r + y)``.
GPU: under bf16 autocast against an fp64 restatement of the same fp32 math (z = r + y with the
16-bit operand widened exactly — rounded to bf16 when both operands are bf16, as autocast's bf16
add is — LayerNorm over the last dim) — outputs, both input gradients
(in their own dtypes) and gamma / beta gradients; fp32 tolerances, bf16 rounding for 16-bit
gradients."""
import pytest
import torch

from conftest import PKG

AN = PKG.models.modules.add_norm
ATT = PKG.models.modules.attention


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
    z = r64 + y64
    if r.dtype == torch.bfloat16 and y.dtype == torch.bfloat16:
        # autocast's bf16 + bf16 add rounds z to bf16 before the fp32 LayerNorm (gradient passes through)
        zr = (r.detach().float() + y.detach().float()).bfloat16().double()
        z = z + (zr - z).detach()
    out = torch.nn.functional.layer_norm(z, (r.shape[-1],), w64, b64, eps)
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
def test_bf16_residual_matches_autocast_composition(dev):
    """Both operands bf16 (the multimodal FFN's residual): the fused kernel reproduces the
    reference's autocast ``norm(r + y)`` (a bf16 add, then the fp32 LayerNorm)."""
    torch.manual_seed(5)
    norm = torch.nn.LayerNorm(512).to(dev)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.5, 0.5)
    r = (torch.randn(4096, 512, device=dev) * 3).bfloat16()
    y = torch.randn(4096, 512, device=dev).bfloat16()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        fused = AN.add_layer_norm(r, y, norm)
        ref = norm(r + y)
    assert ref.dtype == torch.float32
    torch.testing.assert_close(fused, ref, rtol=2e-6, atol=2e-6)


@pytest.mark.gpu
def test_unsupported_width_falls_back(dev):
    norm = torch.nn.LayerNorm(100).to(dev)
    r, y = torch.randn(4, 100, device=dev), torch.randn(4, 100, device=dev).bfloat16()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = AN.add_layer_norm(r, y, norm)
        ref = norm(r + y)
    torch.testing.assert_close(out, ref, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("rows,d,with_pos", [(15360, 512, True), (800, 512, False), (37, 1024, True)])
def test_carry_matches_fp64(dev, rows, d, with_pos):
    """add_layer_norm_carry: out (fp32), out16 = bf16(out), q16 = bf16(out + pos) and, with all three
    gradients given, the input / pos / gamma / beta gradients against fp64."""
    torch.manual_seed(rows)
    norm = torch.nn.LayerNorm(d).to(dev)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.5, 0.5)
    r = torch.randn(rows, d, device=dev).requires_grad_(True)
    y = torch.randn(rows, d, device=dev).bfloat16().requires_grad_(True)
    pos = torch.randn(rows, d, device=dev).requires_grad_(True) if with_pos else None
    g0, g1, g2 = (torch.randn(rows, d, device=dev) for _ in range(3))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out, out16, q16 = AN.add_layer_norm_carry(r, y, norm, pos)
    assert out.dtype == torch.float32 and out16.dtype == torch.bfloat16
    torch.testing.assert_close(out16, out.bfloat16(), rtol=0, atol=0)
    loss = (out * g0).sum() + (out16.float() * g1.bfloat16().float()).sum()
    if with_pos:
        torch.testing.assert_close(q16, (out + pos).bfloat16(), rtol=0, atol=0)
        loss = loss + (q16.float() * g2.bfloat16().float()).sum()
    else:
        assert q16 is None
    loss.backward()
    dout = g0.double() + g1.bfloat16().double() + (g2.bfloat16().double() if with_pos else 0)
    ro, rgr, rgy, rgw, rgb = _ref(r, y, norm.weight, norm.bias, norm.eps, dout)
    torch.testing.assert_close(out.double(), ro, rtol=1e-5, atol=1e-5)
    tol = 2 ** -8
    torch.testing.assert_close(r.grad.double(), rgr, rtol=1e-5, atol=1e-5 * rgr.abs().max().item())
    torch.testing.assert_close(y.grad.double(), rgy, rtol=tol, atol=tol * rgy.abs().max().item())
    torch.testing.assert_close(norm.weight.grad.double(), rgw, rtol=1e-5, atol=1e-5 * rgw.abs().max().item())
    torch.testing.assert_close(norm.bias.grad.double(), rgb, rtol=1e-5, atol=1e-5 * rgb.abs().max().item())
    if with_pos:
        torch.testing.assert_close(pos.grad, g2.bfloat16().float(), rtol=0, atol=0)


@pytest.mark.gpu
def test_carry_only_bf16_gradients(dev):
    """The fp32 output unused (its gradient None): the backward runs on the 16-bit gradients alone."""
    torch.manual_seed(3)
    norm = torch.nn.LayerNorm(512).to(dev)
    r = torch.randn(64, 512, device=dev).requires_grad_(True)
    y = torch.randn(64, 512, device=dev).bfloat16().requires_grad_(True)
    g1 = torch.randn(64, 512, device=dev).bfloat16()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        _, out16, _ = AN.add_layer_norm_carry(r, y, norm)
    (out16.float() * g1.float()).sum().backward()
    ro, rgr, rgy, rgw, rgb = _ref(r, y, norm.weight, norm.bias, norm.eps, g1.double())
    torch.testing.assert_close(r.grad.double(), rgr, rtol=1e-5, atol=1e-5 * rgr.abs().max().item())
    torch.testing.assert_close(norm.bias.grad.double(), rgb, rtol=1e-5, atol=1e-5 * rgb.abs().max().item())


@pytest.mark.gpu
def test_encoder_carry_matches_uncarried(dev, monkeypatch):
    """The encoder stack with carried bf16 operands against the same stack layer by layer (autocast
    casts, pos adds): forward bit-identical (dropout 0: the same bf16 operands), gradients to
    bf16-ulp tolerance elementwise and in norm."""
    UT = PKG.models.deformable.unimodal_deformable_transformer
    torch.manual_seed(0)
    B, shapes, d = 2, [128, 64, 32, 16], 512
    layer = UT.DeformableTransformerEncoderLayer(d, 1024, 0.0, "relu", 4, 8, 4)
    enc = UT.DeformableTransformerEncoder(layer, 3).to(dev)
    S = sum(shapes)
    ts = torch.tensor(shapes, device=dev)
    lsi = torch.cat([ts.new_zeros(1), ts.cumsum(0)[:-1]])
    vr = torch.ones(B, 4, device=dev)
    src0 = torch.randn(B, S, d, device=dev)
    pos0 = torch.randn(B, S, d, device=dev)

    def run():
        enc.zero_grad(set_to_none=True)
        src = src0.clone().requires_grad_(True)
        pos = pos0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = enc(src, ts, lsi, vr, pos=pos)
        (out * torch.linspace(-1, 1, d, device=dev)).sum().backward()
        return out.detach(), src.grad, pos.grad, [p.grad.clone() for p in enc.parameters()]

    o1, gs1, gp1, gw1 = run()
    monkeypatch.setattr(UT, "carry_supported", lambda *a: False)
    o2, gs2, gp2, gw2 = run()
    torch.testing.assert_close(o1, o2, rtol=0, atol=0)
    # the gradients cross bf16 GEMMs and bf16 branch gradients: a different fp32 summation order
    # at the layer boundary moves a few elements by one bf16 ulp of their branch
    for a, b in [(gs1, gs2), (gp1, gp2)] + list(zip(gw1, gw2)):
        torch.testing.assert_close(a, b, rtol=2 ** -7, atol=2 ** -8 * b.abs().max().item())
        assert (a - b).norm() <= 2 ** -8 * b.norm()  # ~one bf16 rounding (2^-9) per branch, two branches


def _mask_of(seed, rows, d, p, dev):
    """The keep mask the kernel draws for (seed, p) on a rows x d call, read back from a forward
    of r = 0, y = 1: kept elements are the ones above their row mean (gamma 1, beta 0)."""
    norm = torch.nn.LayerNorm(d).to(dev)
    r = torch.zeros(rows, d, device=dev)
    y = torch.ones(rows, d, device=dev, dtype=torch.bfloat16)
    out = AN._AddLayerNorm.apply(r, y, norm.weight, norm.bias, norm.eps, p, seed)
    return out > 0


@pytest.mark.gpu
@pytest.mark.parametrize("ydt", [torch.bfloat16, torch.float32])
def test_fused_dropout_matches_fp64_with_its_mask(dev, ydt):
    """norm(r + dropout_p(y)) with the dropout inside the kernel: keep rate ~ 1 - p, and outputs and
    gradients equal the fp64 restatement run with the kernel's own mask (regenerated from the seed
    in the backward: dy is zero exactly where dropped)."""
    rows, d, p = 4096, 512, 0.1
    torch.manual_seed(5)
    seed = torch.tensor([123456789], device=dev, dtype=torch.int64)
    keep = _mask_of(seed, rows, d, p, dev)
    rate = keep.float().mean().item()
    assert abs(rate - (1 - p)) < 0.005, rate
    norm = torch.nn.LayerNorm(d).to(dev)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.5, 0.5)
    r = torch.randn(rows, d, device=dev).requires_grad_(True)
    y = torch.randn(rows, d, device=dev).to(ydt).requires_grad_(True)
    dout = torch.randn(rows, d, device=dev)
    out = AN._AddLayerNorm.apply(r, y, norm.weight, norm.bias, norm.eps, p, seed)
    out.backward(dout)
    yd = (y.detach().float() * keep / (1 - p)).to(ydt)  # ATen's dropout of a bf16 tensor rounds to bf16
    ro, rgr, rgyd, rgw, rgb = _ref(r, yd, norm.weight, norm.bias, norm.eps, dout)
    torch.testing.assert_close(out.double(), ro, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(r.grad.double(), rgr, rtol=1e-5, atol=1e-5 * rgr.abs().max().item())
    rgy = rgyd * keep / (1 - p)
    tol = 2 ** -8 if ydt == torch.bfloat16 else 1e-5
    torch.testing.assert_close(y.grad.double(), rgy, rtol=tol, atol=tol * rgy.abs().max().item())
    assert bool((y.grad[~keep] == 0).all())
    torch.testing.assert_close(norm.weight.grad.double(), rgw, rtol=1e-5, atol=1e-5 * rgw.abs().max().item())
    # another seed, another mask; the carry variant draws the same mask from the same seed
    other = _mask_of(torch.tensor([987654321], device=dev, dtype=torch.int64), rows, d, p, dev)
    assert (other != keep).float().mean().item() > 0.1
    with torch.no_grad():
        o2, _, _ = AN._AddLayerNormCarry.apply(r, y, norm.weight, norm.bias, None, norm.eps, p, seed)
    torch.testing.assert_close(o2, out.detach(), rtol=0, atol=0)


@pytest.mark.gpu
def test_dropout_module_routes_through_kernel(dev):
    """add_layer_norm(..., dropout=nn.Dropout) in training draws a fresh seed per call (different
    masks), and in eval mode is exactly norm(r + y)."""
    torch.manual_seed(0)
    norm = torch.nn.LayerNorm(512).to(dev)
    drop = torch.nn.Dropout(0.1)
    r = torch.randn(256, 512, device=dev)
    y = torch.randn(256, 512, device=dev).bfloat16()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        a = AN.add_layer_norm(r, y, norm, dropout=drop)
        b = AN.add_layer_norm(r, y, norm, dropout=drop)
        drop.eval()
        c = AN.add_layer_norm(r, y, norm, dropout=drop)
        e = AN.add_layer_norm(r, y, norm)
    assert not torch.equal(a, b)
    torch.testing.assert_close(c, e, rtol=0, atol=0)


@pytest.mark.gpu
def test_decoder_carry_matches_uncarried(dev, monkeypatch):
    """Decoder layers with the cross-attention query bf16(tgt + query_pos) and the linear1 operand
    bf16(tgt) from the fused add + LayerNorms, against the uncarried layers: forward bit-identical
    (dropout 0), gradients (memory, tgt, query_pos, parameters) to bf16-ulp tolerance."""
    UT = PKG.models.deformable.unimodal_deformable_transformer
    torch.manual_seed(1)
    B, Q, shapes, d = 2, 100, [128, 64, 32, 16], 512
    layer = UT.DeformableTransformerDecoderLayer(d, 1024, 0.0, "relu", 4, 8, 4)
    dec = UT.DeformableTransformerDecoder(layer, 2, return_intermediate=True).to(dev)
    S = sum(shapes)
    ts = torch.tensor(shapes, device=dev)
    lsi = torch.cat([ts.new_zeros(1), ts.cumsum(0)[:-1]])
    vr = torch.ones(B, 4, device=dev)
    mem0 = torch.randn(B, S, d, device=dev)
    tgt0 = torch.randn(B, Q, d, device=dev)
    qpos0 = torch.randn(Q, d, device=dev)
    ref = torch.rand(B, Q, 1, device=dev)
    qmask = torch.ones(B, Q, dtype=torch.bool, device=dev)

    def run():
        dec.zero_grad(set_to_none=True)
        mem, tgt = mem0.clone().requires_grad_(True), tgt0.clone().requires_grad_(True)
        qpos = qpos0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            hs, _ = dec(tgt, ref, mem, ts, lsi, vr, query_pos=qpos.unsqueeze(0).expand(B, -1, -1),
                        query_padding_mask=qmask)
        (hs.float() * torch.linspace(-1, 1, d, device=dev)).sum().backward()
        return hs.detach(), [mem.grad, tgt.grad, qpos.grad] + [p.grad.clone() for p in dec.parameters()]

    h1, g1 = run()
    monkeypatch.setattr(UT, "carry_supported", lambda *a: False)
    h2, g2 = run()
    torch.testing.assert_close(h1, h2, rtol=0, atol=0)
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=2 ** -7, atol=2 ** -8 * b.abs().max().item())
        assert (a - b).norm() <= 2 ** -8 * b.norm()


@pytest.mark.gpu
def test_multimodal_layer_carry_matches_uncarried(dev, monkeypatch):
    """Multimodal encoder layer whose self blocks hand the cross-modal MSDA calls bf16(out) from the
    fused add + LayerNorm, against the same layer with the fp32 output (autocast casts it per call):
    forward bit-identical (dropout 0), gradients to bf16-ulp tolerance.

    Gradient bounds: 2^-7 of the norm, 2^-6 of the max element-wise.  Each path's gradient carries its
    own bf16 rounding noise; against an fp64 truth of this layer (tools/mm_layer_dense_diag.py, run
    r06o) the carried, uncarried, dense and non-dense runs are equally accurate (attention_weights
    gradients 1.0e-2 off in norm for every one, the worst attention_weights.bias element 2.8-3.1 off
    a max of 504), so two such paths differ by up to twice one path's error: 4.6 (0.9 % of the max)
    at one bias element with the dense small-pyramid kernels, above the 2^-7 element bound."""
    MT = PKG.models.deformable.multimodal_deformable_transformer
    torch.manual_seed(2)
    B, d, vs, as_ = 2, 512, [128, 64, 32, 16], [50, 25, 13, 7]
    layer = MT.MultimodalDeformableTransformerEncoderLayer(d, 1024, 0.0, "relu", 4, 8, 4).to(dev)

    def meta(shapes):
        ts = torch.tensor(shapes, device=dev)
        return ts, torch.cat([ts.new_zeros(1), ts.cumsum(0)[:-1]])
    vts, vlsi = meta(vs)
    ats, alsi = meta(as_)
    ones = torch.ones(B, 4, device=dev)
    vref = MT.MultimodalDeformableTransformerEncoder.get_reference_points(vts, ones, dev)
    aref = MT.MultimodalDeformableTransformerEncoder.get_reference_points(ats, ones, dev)
    v0, a0 = torch.randn(B, sum(vs), d, device=dev), torch.randn(B, sum(as_), d, device=dev)
    vp0, ap0 = torch.randn(B, sum(vs), d, device=dev), torch.randn(B, sum(as_), d, device=dev)
    wv, wa = torch.randn(d, device=dev), torch.randn(d, device=dev)

    def run():
        layer.zero_grad(set_to_none=True)
        v, a = v0.clone().requires_grad_(True), a0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ov, oa = layer(v, vp0, vref, vts, vlsi, None, a, ap0, aref, ats, alsi, None)
        # weighted: a plain sum of LayerNorm outputs has ~zero gradient (rounding noise only)
        (ov.float() * wv).sum().add_((oa.float() * wa).sum()).backward()
        return (ov.detach(), oa.detach()), [v.grad, a.grad] + [p.grad.clone() for p in layer.parameters()]

    o1, g1 = run()
    AN_ = PKG.models.modules.add_norm

    def uncarried(r, y, norm, pos=None, dropout=None):
        out = AN_.add_layer_norm(r, y, norm, dropout)
        return out, out, None
    monkeypatch.setattr(MT, "add_layer_norm_carry", uncarried)
    o2, g2 = run()
    for a, b in zip(o1, o2):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=2 ** -7, atol=2 ** -6 * b.abs().max().item())
        # the FFN residual add is bf16 + bf16 (rounded to bf16 as autocast's add): one more bf16
        # rounding on both paths, so the carried / uncarried gradient noise is ~2^-8 of the norm
        assert (a - b).norm() <= 2 ** -7 * b.norm()


@pytest.mark.gpu
def test_multimodal_encoder_carry_matches_uncarried(dev, monkeypatch):
    """Multimodal encoder stack carrying (src, bf16 src, bf16 src + pos) per stream between layers,
    against the layer-by-layer stack: forward bit-identical (dropout 0).  Gradients (both inputs,
    both positional embeddings, parameters) cross 3 layers of bf16 GEMMs and cross-modal MSDA, so
    both bf16 runs are held to the fp32 run of the same stack: the carried one may not be further
    from it than the uncarried one (x1.25), and the two agree to bf16-ulp tolerance elementwise."""
    MT = PKG.models.deformable.multimodal_deformable_transformer
    torch.manual_seed(3)
    B, d, vs, as_ = 2, 512, [128, 64, 32, 16], [50, 25, 13, 7]
    layer = MT.MultimodalDeformableTransformerEncoderLayer(d, 1024, 0.0, "relu", 4, 8, 4)
    enc = MT.MultimodalDeformableTransformerEncoder(layer, 3).to(dev)

    def meta(shapes):
        ts = torch.tensor(shapes, device=dev)
        return ts, torch.cat([ts.new_zeros(1), ts.cumsum(0)[:-1]])
    vts, vlsi = meta(vs)
    ats, alsi = meta(as_)
    ones = torch.ones(B, 4, device=dev)
    v0, a0 = torch.randn(B, sum(vs), d, device=dev), torch.randn(B, sum(as_), d, device=dev)
    vp0, ap0 = torch.randn(B, sum(vs), d, device=dev), torch.randn(B, sum(as_), d, device=dev)
    wv, wa = torch.randn(d, device=dev), torch.randn(d, device=dev)

    def run(amp=True):
        enc.zero_grad(set_to_none=True)
        v, a = v0.clone().requires_grad_(True), a0.clone().requires_grad_(True)
        vp, ap = vp0.clone().requires_grad_(True), ap0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            ov, oa = enc(v, vts, vlsi, ones, vp, None, a, ats, alsi, ones, ap, None)
        # weighted: a plain sum of LayerNorm outputs has ~zero gradient (rounding noise only)
        (ov.float() * wv).sum().add_((oa.float() * wa).sum()).backward()
        return (ov.detach(), oa.detach()), [v.grad, a.grad, vp.grad, ap.grad] + [
            p.grad.clone() for p in enc.parameters()]

    monkeypatch.setenv("MFL_MM_JOINT", "0")  # the per-stream carried layers (the joint rows: the next test)
    o1, g1 = run()
    monkeypatch.setattr(MT, "carry_supported", lambda *a: False)
    o2, g2 = run()
    _, g3 = run(amp=False)
    for a, b in zip(o1, o2):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    for a, b, c in zip(g1, g2, g3):
        torch.testing.assert_close(a, b, rtol=2 ** -7, atol=2 ** -7 * b.abs().max().item())
        assert (a - c).norm() <= 1.25 * (b - c).norm() + 1e-6 * c.norm()


@pytest.mark.gpu
def test_multimodal_encoder_joint_rows_match_per_stream(dev, monkeypatch):
    """The multimodal encoder on joint rows (MultimodalDeformableTransformerEncoder._forward_joint: both
    streams' rows in one tensor; per layer ONE value / query / output projection of the shared self_attn
    for the two self calls and ONE for the two cross-modal calls, one MSDA launch per call, the add +
    LayerNorms and the FFN once over all rows) against the per-stream carried layers.  A GEMM over more
    rows may pick another kernel (another bf16 rounding), so both are held to the fp32 run of the same
    stack: outputs and gradients (inputs, positional embeddings, every parameter) no further from it than
    the per-stream path (x1.25), and the two within bf16-ulp tolerance of each other; the joint path's
    launches asserted by trace."""
    MT = PKG.models.deformable.multimodal_deformable_transformer
    torch.manual_seed(4)
    B, d, vs, as_ = 2, 512, [128, 64, 32, 16], [50, 25, 13, 7]
    layer = MT.MultimodalDeformableTransformerEncoderLayer(d, 1024, 0.0, "relu", 4, 8, 4)
    enc = MT.MultimodalDeformableTransformerEncoder(layer, 3).to(dev)

    def meta(shapes):
        ts = torch.tensor(shapes, device=dev)
        return ts, torch.cat([ts.new_zeros(1), ts.cumsum(0)[:-1]])
    vts, vlsi = meta(vs)
    ats, alsi = meta(as_)
    ones = torch.ones(B, 4, device=dev)
    v0, a0 = torch.randn(B, sum(vs), d, device=dev), torch.randn(B, sum(as_), d, device=dev)
    vp0, ap0 = torch.randn(B, sum(vs), d, device=dev), torch.randn(B, sum(as_), d, device=dev)
    vmask = torch.zeros(B, sum(vs), dtype=torch.bool, device=dev)
    amask = torch.zeros(B, sum(as_), dtype=torch.bool, device=dev)
    for l, (t, s0) in enumerate(zip(vs, vlsi.tolist())):
        vmask[1, s0 + (3 * t) // 4:s0 + t] = True
    for l, (t, s0) in enumerate(zip(as_, alsi.tolist())):
        amask[1, s0 + (3 * t) // 4:s0 + t] = True
    vr = torch.tensor([[1.0] * 4, [0.75] * 4], device=dev)
    wv, wa = torch.randn(d, device=dev), torch.randn(d, device=dev)

    def run(amp=True):
        enc.zero_grad(set_to_none=True)
        v, a = v0.clone().requires_grad_(True), a0.clone().requires_grad_(True)
        vp, ap = vp0.clone().requires_grad_(True), ap0.clone().requires_grad_(True)
        PKG._trace.clear()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            ov, oa = enc(v, vts, vlsi, vr, vp, vmask, a, ats, alsi, vr, ap, amask)
        hits = dict(PKG._trace.hits)
        (ov.float() * wv).sum().add_((oa.float() * wa).sum()).backward()
        return [ov.detach().float(), oa.detach().float()], [v.grad, a.grad, vp.grad, ap.grad] + [
            p.grad.clone() for p in enc.parameters()], hits

    o1, g1, hits = run()
    assert hits.get("msda_joint", 0) == 6 and hits.get("query_prologue_joint", 0) == 6, hits
    monkeypatch.setenv("MFL_MM_JOINT", "0")
    o2, g2, hits2 = run()
    assert hits2.get("msda_joint", 0) == 0, hits2
    o3, g3, _ = run(amp=False)
    for a, b, c in zip(o1 + g1, o2 + g2, o3 + g3):
        torch.testing.assert_close(a, b, rtol=2 ** -6, atol=2 ** -6 * b.abs().max().item())
        assert (a - c).norm() <= 1.25 * (b - c).norm() + 1e-6 * c.norm()


@pytest.mark.gpu
def test_decoder_self_attention_carry_matches_uncarried(dev, monkeypatch):
    """Decoder stack whose layers hand the next layer's self-attention its bf16 inputs
    (bf16(out), bf16(out + query_pos)) from the last fused add + LayerNorm, against the same stack
    casting them in each layer: forward bit-identical (dropout 0), gradients to fp32-sum order."""
    UT = PKG.models.deformable.unimodal_deformable_transformer
    torch.manual_seed(6)
    layer = UT.DeformableTransformerDecoderLayer(512, 1024, 0.0, "relu", 4, 8, 4)
    dec = UT.DeformableTransformerDecoder(layer, 3, return_intermediate=True).to(dev)
    shapes = [256, 128, 64, 32]
    ts = torch.tensor(shapes, device=dev)
    lsi = torch.cat([ts.new_zeros(1), ts.cumsum(0)[:-1]])
    B, Q = 2, 100
    src = torch.randn(B, sum(shapes), 512, device=dev)
    tgt0 = torch.randn(B, Q, 512, device=dev)
    qpos = torch.randn(B, Q, 512, device=dev, requires_grad=True)
    ref = torch.rand(B, Q, 1, device=dev)
    vr = torch.ones(B, 4, device=dev)
    qmask = torch.ones(B, Q, dtype=torch.bool, device=dev)
    w = torch.randn(512, device=dev)

    def run():
        dec.zero_grad(set_to_none=True)
        qpos.grad = None
        tgt = tgt0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            hs, _ = dec(tgt, ref, src, ts, lsi, vr, qpos, None, qmask)
        (hs.float() * w).sum().backward()
        return hs.detach(), [tgt.grad, qpos.grad] + [p.grad.clone() for p in dec.parameters() if p.grad is not None]

    h1, g1 = run()
    real = ATT.mha_self_attention
    monkeypatch.setattr(UT, "mha_self_attention", lambda m, t, p, q, carried=None: real(m, t, p, q))
    h2, g2 = run()
    torch.testing.assert_close(h1, h2, rtol=0, atol=0)
    assert len(g1) == len(g2)
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-3 * b.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("rows,d", [(15360, 512), (800, 512), (37, 1024)])
def test_backward_ex2_dy_colsum_and_pos_accumulation(dev, rows, d):
    """mfl_add_layernorm_backward_ex2: dy_colsum = the column sums of dy as stored (the producing
    Linear's bias gradient, handed to it by add_norm._attach_colsum) and dpos_accumulate adds dq16 into
    dpos (a pos shared by several layers: add_norm.pos_sink) — the other outputs as the _ex entry's."""
    lib = PKG._native.load_library()
    torch.manual_seed(3)
    norm = torch.nn.LayerNorm(d).to(dev)
    r = torch.randn(rows, d, device=dev)
    y = torch.randn(rows, d, device=dev).bfloat16()
    dout = torch.randn(rows, d, device=dev)
    dq16 = torch.randn(rows, d, device=dev).bfloat16()
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    out = torch.empty(rows, d, device=dev)
    sh = PKG._native.stream_handle(dev)
    assert lib.mfl_add_layernorm_forward(r.data_ptr(), 0, y.data_ptr(), 2, norm.weight.data_ptr(), norm.bias.data_ptr(),
                                         rows, d, norm.eps, out.data_ptr(), mean.data_ptr(), rstd.data_ptr(), sh) == 0
    ws = torch.empty(lib.mfl_add_layernorm_workspace_bytes(rows, d), dtype=torch.uint8, device=dev)

    def call(fn_ex2, dpos, acc, colsum):
        dr, dy = torch.empty_like(r), torch.empty_like(y)
        dw, db = torch.empty(d, device=dev), torch.empty(d, device=dev)
        args = (dout.data_ptr(), None, dq16.data_ptr(), r.data_ptr(), 0, y.data_ptr(), 2, norm.weight.data_ptr(),
                mean.data_ptr(), rstd.data_ptr(), rows, d, dr.data_ptr(), dy.data_ptr(), dw.data_ptr(), db.data_ptr(),
                dpos.data_ptr())
        if fn_ex2:
            rc = lib.mfl_add_layernorm_backward_ex2(*args, acc, None if colsum is None else colsum.data_ptr(), 0.0,
                                                    None, ws.data_ptr(), sh)
        else:
            rc = lib.mfl_add_layernorm_backward_ex(*args, 0.0, None, ws.data_ptr(), sh)
        assert rc == 0, lib.mfl_add_layernorm_last_error()
        return dr, dy, dw, db

    dpos_ref = torch.empty(rows, d, device=dev)
    ref = call(False, dpos_ref, 0, None)
    dpos = torch.full((rows, d), 0.25, device=dev)
    colsum = torch.empty(d, device=dev)
    got = call(True, dpos, 1, colsum)
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    torch.testing.assert_close(dpos, dq16.float() + 0.25, rtol=0, atol=0)
    want = got[1].double().sum(0)
    torch.testing.assert_close(colsum.double(), want, rtol=1e-5, atol=1e-5 * want.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("with_acc", [False, True])
def test_carry_entry_matches_composition(dev, with_acc):
    """add_norm.carry_entry (csrc/add_layernorm.hip carry_entry_*): (src, bf16(src), bf16(src + pos))
    are autocast's casts of the reference's with_pos_embed (unimodal_deformable_transformer.py:241)
    bit for bit; src's gradient is the sum of its three gradients, pos's the query's (also through a
    pos_sink accumulator shared with another consumer)."""
    g = torch.Generator(device=dev).manual_seed(3)
    shape = (4, 960, 512)
    src = torch.randn(shape, device=dev, generator=g, requires_grad=True)
    pos0 = torch.randn(shape, device=dev, generator=g, requires_grad=True)
    dr, dv, dq = (torch.randn(shape, device=dev, generator=g) for _ in range(3))
    dv, dq = dv.bfloat16(), dq.bfloat16()
    extra = torch.randn(shape, device=dev, generator=g)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        pos, acc = AN.pos_sink(pos0) if with_acc else (pos0, None)
        PKG._trace.clear()
        r, v16, q16 = AN.carry_entry(src, pos, acc)
        assert PKG._trace.hits.get("carry_entry", 0) == 1
        other = (pos * 2.0).sum() if with_acc else None  # another consumer of pos (autograd's gradient)
    assert torch.equal(v16, src.detach().bfloat16()) and torch.equal(q16, (src.detach() + pos0.detach()).bfloat16())
    loss = (r * dr).sum() + (v16.float() * dv.float()).sum() + (q16.float() * dq.float()).sum()
    if other is not None:
        loss = loss + other
    gs, gp = torch.autograd.grad(loss, [src, pos0])
    torch.testing.assert_close(gs, dr + dv.float() + dq.float(), rtol=1e-6, atol=1e-6)
    want_p = dq.float() + (2.0 if with_acc else 0.0)
    torch.testing.assert_close(gp, want_p, rtol=1e-6, atol=1e-6)
    del extra


@pytest.mark.gpu
def test_multimodal_decoder_carry_matches_uncarried(dev, monkeypatch):
    """Multimodal decoder stack with the bf16 operands carried between its fused add + LayerNorms
    (MultimodalDeformableTransformerDecoderLayer.forward_carry: one bf16(tgt + query_pos) for both
    cross-attentions, query_pos's gradient summed in place) against the layer-by-layer stack: forward
    bit-identical (dropout 0); gradients held to the fp32 run as in the encoder test above."""
    MT = PKG.models.deformable.multimodal_deformable_transformer
    torch.manual_seed(5)
    B, d, Q, vs, as_ = 2, 512, 30, [128, 64, 32, 16], [50, 25, 13, 7]
    layer = MT.MultimodalDeformableTransformerDecoderLayer(d, 1024, 0.0, "relu", 4, 8, 4)
    dec = MT.MultimodalDeformableTransformerDecoder(layer, 3, return_intermediate=True).to(dev)

    def meta(shapes):
        ts = torch.tensor(shapes, device=dev)
        return ts, torch.cat([ts.new_zeros(1), ts.cumsum(0)[:-1]])
    vts, vlsi = meta(vs)
    ats, alsi = meta(as_)
    ones = torch.ones(B, 4, device=dev)
    t0, qp0 = torch.randn(B, Q, d, device=dev), torch.randn(B, Q, d, device=dev)
    ref = torch.rand(B, Q, 1, device=dev)
    qmask = torch.ones(B, Q, dtype=torch.bool, device=dev)
    mv0, ma0 = torch.randn(B, sum(vs), d, device=dev), torch.randn(B, sum(as_), d, device=dev)
    w = torch.randn(d, device=dev)

    def run(amp=True):
        dec.zero_grad(set_to_none=True)
        t, qp = t0.clone().requires_grad_(True), qp0.clone().requires_grad_(True)
        mv, ma = mv0.clone().requires_grad_(True), ma0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            hs, _ = dec(t, ref, qp, qmask, mv, vts, vlsi, ones, None, ma, ats, alsi, ones, None)
        (hs.float() * w).sum().backward()
        return hs.detach(), [t.grad, qp.grad, mv.grad, ma.grad] + [p.grad.clone() for p in dec.parameters()
                                                                   if p.grad is not None]

    PKG._trace.clear()
    o1, g1 = run()
    assert PKG._trace.hits.get("add_ln_carry", 0) >= 6  # two carried add + LayerNorms per layer
    monkeypatch.setattr(MT, "carry_supported", lambda *a: False)
    o2, g2 = run()
    _, g3 = run(amp=False)
    torch.testing.assert_close(o1, o2, rtol=0, atol=0)
    assert len(g1) == len(g2) == len(g3)
    for a, b, c in zip(g1, g2, g3):
        torch.testing.assert_close(a, b, rtol=2 ** -7, atol=2 ** -7 * b.abs().max().item())
        assert (a - c).norm() <= 1.25 * (b - c).norm() + 1e-6 * c.norm()
