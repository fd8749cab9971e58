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
    N, S, C = 3, (1001 if kind == "tail" else 1920), 512  # (1001: rows not a multiple of a wave's 64)
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
    g0 = g.clone()
    out.backward(g)
    torch.testing.assert_close(x.grad, g.masked_fill(mask[..., None], 0.0), rtol=0, atol=0)
    assert torch.equal(g, g0)  # a gradient the caller holds is not written in place


@pytest.mark.gpu
def test_zero_rows_backward_in_place_only_on_private_msda_gradient(dev, monkeypatch):
    """The backward zeroes in place only the gradient the MSDA backward allocated (tagged); a
    second consumer of the masked value makes autograd hand over a fresh sum instead, which is
    zeroed out of place — both give masked_fill's gradient."""
    torch.manual_seed(3)
    shapes, B, M, D, Lq, P = [32, 16, 8, 4], 2, 4, 16, 12, 4
    S = sum(shapes)
    mask = torch.rand(B, S, device=dev) < 0.3
    loc = torch.rand(B, Lq, M, 4, P, device=dev)
    aw = torch.rand(B, Lq, M, 4, P, device=dev)
    gout = torch.randn(B, Lq, M * D, device=dev)
    starts = [0, 32, 48, 56]
    inplace = []
    real = ATT._zero_rows
    monkeypatch.setattr(ATT, "_zero_rows", lambda x, m: inplace.append(x.data_ptr()) or real(x, m))
    for second in (False, True):
        x = torch.randn(B, S, M * D, device=dev, requires_grad=True)
        inplace.clear()
        v = ATT.mask_padding_rows(x * 1, mask)
        out = PKG.msda.msda_apply(v.view(B, S, M, D), shapes, starts, loc, aw)
        loss = (out * gout).sum() + ((v * 3).sum() if second else 0)
        loss.backward()
        xr = x.detach().clone().requires_grad_(True)
        vr = (xr * 1).masked_fill(mask[..., None], 0.0)
        outr = PKG.msda.msda_apply(vr.view(B, S, M, D), shapes, starts, loc, aw)
        ((outr * gout).sum() + ((vr * 3).sum() if second else 0)).backward()
        torch.testing.assert_close(x.grad, xr.grad, rtol=0, atol=0)
        # forward zeroing, plus the backward's in place only for the MSDA backward's own gradient
        assert len(inplace) == (1 if second else 2)


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


@pytest.mark.gpu
@pytest.mark.parametrize("carried,padded", [(False, False), (True, True), (False, True)])
def test_layer_values_match_per_layer_projections(dev, carried, padded):
    """The decoder's value projections of all layers as one batched GEMM each way
    (models/modules/value_proj.py) against each layer's own ``value_proj(src).masked_fill(...)``
    (reference attention.py:461-463) under bf16 autocast: values to bf16 rounding of the same
    fp32-accumulated product, gradients of src / weights / biases to bf16-GEMM tolerance."""
    VP = PKG.models.modules.value_proj
    torch.manual_seed(3)
    n, B, S, C = 4, 2, 1920, 512
    attns = [ATT.MSDeformAttn(C, 4, 8, 4).to(dev) for _ in range(n)]
    for a in attns:
        torch.nn.init.normal_(a.value_proj.bias, std=0.5)
    src0 = torch.randn(B, S, C, device=dev)
    mask = (torch.rand(B, S, device=dev) < 0.2) if padded else None
    gs = [torch.randn(B, S, C, device=dev).bfloat16() for _ in range(n)]

    def run(batched):
        for a in attns:
            a.zero_grad(set_to_none=True)
        src = src0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            x = src
            if carried:
                x16 = src.bfloat16()
                x = src * 1
                x._mfl_bf16 = x16
            if batched:
                assert VP.layer_values_supported(attns, x, mask)
                vals = VP.layer_values(attns, x, mask)
            else:
                vals = [a.value_proj(x) for a in attns]
                if mask is not None:
                    vals = [v.masked_fill(mask[..., None], 0.0) for v in vals]
        sum((v.float() * g.float()).sum() for v, g in zip(vals, gs)).backward()
        return vals, [src.grad] + [p.grad for a in attns for p in (a.value_proj.weight, a.value_proj.bias)]

    v1, g1 = run(True)
    v0, g0 = run(False)
    for a, b in zip(v1, v0):
        assert a.dtype == torch.bfloat16
        torch.testing.assert_close(a.float(), b.float(), rtol=2 ** -7, atol=2 ** -7)
        if mask is not None:
            assert (a[mask] == 0).all()
    for a, b in zip(g1, g0):
        torch.testing.assert_close(a.float(), b.float(), rtol=2 ** -6, atol=2 ** -6 * b.abs().max().item())


@pytest.mark.gpu
def test_mha_self_attention_autocast_matches_module(dev):
    """The decoder's query self-attention under bf16 autocast (SDPA + the autocast-Linear
    projections, attention.py::mha_self_attention) against nn.MultiheadAttention's own call
    (reference unimodal_deformable_transformer.py:352-353) under the same autocast: output and
    gradients of the input, in_proj and out_proj to bf16 tolerance."""
    torch.manual_seed(4)
    mha = torch.nn.MultiheadAttention(512, 8, dropout=0.0).to(dev)
    tgt0 = torch.randn(8, 100, 512, device=dev)
    pos = torch.randn(8, 100, 512, device=dev)
    qmask = torch.ones(8, 100, dtype=torch.bool, device=dev)
    qmask[3, 90:] = False
    g = torch.randn(8, 100, 512, device=dev)

    def run(mine):
        mha.zero_grad(set_to_none=True)
        tgt = tgt0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if mine:
                out = ATT.mha_self_attention(mha, tgt, pos, qmask)
            else:
                qk = (tgt + pos).transpose(0, 1)
                out = mha(qk, qk, tgt.transpose(0, 1), key_padding_mask=~qmask)[0].transpose(0, 1)
        (out.float() * g).sum().backward()
        return [out.float(), tgt.grad] + [p.grad.float() for p in mha.parameters()]

    for a, b in zip(run(True), run(False)):
        torch.testing.assert_close(a, b, rtol=3e-2, atol=3e-2 * b.abs().max().item())


@pytest.mark.gpu
def test_base_encoder_gemm_convs_match_fp64_and_are_reproducible(dev):
    """BaseEncoder under bf16 autocast runs its Conv1d layers as GEMMs on channels-last rows
    (models/base_encoder.py): outputs and gradients against the module in fp64 within bf16
    tolerance, and two runs bitwise equal (MIOpen's bf16 convolution forward was not:
    tools/determinism_diag.py)."""
    torch.manual_seed(3)
    B, T, d = 4, 128, 256
    enc = PKG.models.base_encoder.BaseEncoder(4, d, d).to(dev)
    pos = PKG.models.modules.embedding_layers.PositionEmbeddingVideoSine(d // 2, normalize=True).to(dev)
    x = torch.randn(B, T, d, device=dev)
    mask = torch.zeros(B, T, dtype=torch.bool, device=dev)
    mask[1, 100:] = True
    dur = torch.tensor([30.0, 60.0, 90.0, 120.0], device=dev)
    gs = [torch.randn(B, d, T >> l, device=dev) for l in range(4)]

    def run(model, xx, autocast):
        xx = xx.detach().clone().requires_grad_(True)
        model.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            srcs, masks, _ = model(xx, mask, dur, pos)
        sum((s.double() * g.double()).sum() for s, g in zip(srcs, gs)).backward()
        return [s.detach().double() for s in srcs] + [xx.grad.double()] + [p.grad.double() for p in model.parameters()]

    a, b = run(enc, x, True), run(enc, x, True)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
    import copy
    # the fp64 reference on the host (reference base_encoder.py:49-89 as the module computes it)
    cpu = torch.device("cpu")
    enc64, pos64 = copy.deepcopy(enc).to(cpu).double(), copy.deepcopy(pos).to(cpu)
    x64, m64, d64 = x.to(cpu).double().requires_grad_(True), mask.to(cpu), dur.to(cpu)
    srcs64, _, _ = enc64(x64, m64, d64, pos64)
    sum((s * g.to(cpu).double()).sum() for s, g in zip(srcs64, gs)).backward()
    ref = [t.detach() for t in srcs64] + [x64.grad] + [p.grad for p in enc64.parameters()]
    a = [t.cpu() for t in a]
    for i, (u, v) in enumerate(zip(a, ref)):
        err = ((u - v).norm() / v.norm().clamp_min(1e-30)).item()
        assert err < 2e-2, (i, err)


@pytest.mark.gpu
def test_linear_group_matches_separate_projections(dev, monkeypatch):
    """value_proj.linear_group (the caption decoder's grouped key / value projections of the clip
    memory and its self-attention q / k / v): outputs and every gradient against the same Linear
    layers applied one by one under bf16 autocast (MFL_LINEAR_GROUP=0): outputs bit for bit (each
    output column is its own fp32-accumulated product, one rounding), gradients to bf16 / fp32
    summation order."""
    torch.manual_seed(4)
    lins = torch.nn.ModuleList([PKG.models.modules.linear.Linear(512, 512) for _ in range(5)]).to(dev)
    x = torch.randn(3, 700, 512, device=dev)
    gs = [torch.randn(3, 700, 512, device=dev) for _ in lins]
    runs = []
    for grouped in (True, False):
        lins.zero_grad()
        xx = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            outs = (PKG.models.modules.value_proj.linear_group(list(lins), xx) if grouped
                    else [lin(xx) for lin in lins])
        sum((o.float() * g).sum() for o, g in zip(outs, gs)).backward()
        runs.append(([o.detach() for o in outs], xx.grad, [p.grad.clone() for p in lins.parameters()]))
    for a, b in zip(runs[0][0], runs[1][0]):
        assert torch.equal(a, b)
    torch.testing.assert_close(runs[0][1], runs[1][1], rtol=2e-2, atol=2e-2)
    for a, b in zip(runs[0][2], runs[1][2]):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-3)


@pytest.mark.gpu
def test_host_weights_never_reach_native_kernels(dev):
    """A Linear / LayerNorm left on the host with a GPU input under bf16 autocast raises torch's
    device-mismatch error instead of handing host pointers to a HIP kernel (the guards in
    linear.py small_addmm / Linear._autocast_dtype and add_norm.py: an earlier version of
    test_base_encoder_gemm_convs_match_fp64_and_are_reproducible built its position embedding on
    the host and the short-M GEMM read the host weight's address)."""
    lin = PKG.models.modules.linear.Linear(128, 128)
    x = torch.randn(64, 128, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        with pytest.raises(RuntimeError):
            lin(x)
    w = torch.randn(128, 128, dtype=torch.bfloat16)
    assert PKG.models.modules.linear.small_addmm(None, x.to(torch.bfloat16), w) is None
    norm = torch.nn.LayerNorm(256)
    r = torch.randn(4, 256, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        with pytest.raises(RuntimeError):
            PKG.models.modules.add_norm.add_layer_norm(r, r, norm)


@pytest.mark.gpu
@pytest.mark.parametrize("T", [(1024, 512, 256, 128), (50, 25, 13, 7)])
def test_level_pos_flatten_matches_reference(dev, T):
    """models/modules/pyramid.py (mfl_level_pos_flatten / mfl_level_colsum): the flattened level
    position embedding of prepare_encoder_inputs (reference unimodal_deformable_transformer.py:90-134)
    is the reference composition bit for bit; its gradients are the reference's (the position
    embeddings' exactly, the level embedding's per-level column sums up to fp32 summation order)."""
    pyr = PKG.models.modules.pyramid
    g = torch.Generator(device=dev).manual_seed(11)
    B, N = 3, 512
    # level 1 as the position embedding returns it: a transposed view of (B, T, N) rows
    leaves = [torch.randn((B, t, N) if i == 1 else (B, N, t), device=dev, generator=g, requires_grad=True)
              for i, t in enumerate(T)]
    poses = [x.transpose(1, 2) if i == 1 else x for i, x in enumerate(leaves)]
    emb = torch.randn(len(T), N, device=dev, generator=g, requires_grad=True)
    go = torch.randn(B, sum(T), N, device=dev, generator=g)
    PKG._trace.clear()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = pyr.level_pos_flatten(poses, emb)
    assert PKG._trace.hits.get("level_pos_flatten", 0) == 1
    ref = pyr._reference(poses, emb)
    assert torch.equal(out, ref)
    got = torch.autograd.grad(out, [emb] + leaves, go)
    want = torch.autograd.grad(ref, [emb] + leaves, go)
    torch.testing.assert_close(got[0], want[0], rtol=1e-5, atol=1e-4)
    for a, b in zip(got[1:], want[1:]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("normalize", [True, False])
def test_pyramid_pos_matches_per_level_embeddings(dev, normalize):
    """pyramid.LevelPositions + mfl_pyramid_pos_flatten: the flattened level position embedding of a
    padded pyramid written from its masks and durations in one kernel equals the reference chain —
    PositionEmbeddingVideoSine per level (embedding_layers.py:185-227, sin / cos of the normalised
    mask cumsum, the duration embedding) cast and flattened with level_embed
    (unimodal_deformable_transformer.py:90-134) — and so do the level_embed and duration-embedding
    gradients."""
    torch.manual_seed(13)
    emb_mod = PKG.models.modules.embedding_layers.PositionEmbeddingVideoSine(256, normalize=normalize).to(dev)
    pyr = PKG.models.modules.pyramid
    B, Ts = 3, (96, 48, 24, 12)
    lens = torch.tensor([96, 70, 31], device=dev)
    masks = [(torch.arange(T, device=dev)[None] * 96 // T) >= lens[:, None] for T in Ts]
    duration = torch.tensor([40.0, 100.0, 3.0], device=dev)
    srcs = [torch.zeros(B, 512, T, device=dev) for T in Ts]
    level_embed = torch.randn(len(Ts), 512, device=dev, requires_grad=True)
    go = torch.randn(B, sum(Ts), 512, device=dev)

    def run(fused):
        emb_mod.zero_grad(set_to_none=True)
        level_embed.grad = None
        lp = pyr.LevelPositions(emb_mod, srcs, masks, duration, [torch.float32] * len(Ts))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            # (the model builds its positions under autocast: the duration embedding's Linear in bf16)
            if not fused:
                list(lp)  # materialise: the per-level reference chain
            PKG._trace.clear()
            out = pyr.level_pos_flatten(lp, level_embed)
        assert (PKG._trace.hits.get("pyramid_pos", 0) == 1) == fused
        (out * go).sum().backward()
        return out.detach(), level_embed.grad.clone(), emb_mod.duration_embed_layer.weight.grad.clone()

    o1, l1, w1 = run(True)
    o2, l2, w2 = run(False)
    torch.testing.assert_close(o1, o2, rtol=2e-6, atol=2e-6)
    torch.testing.assert_close(l1, l2, rtol=1e-5, atol=1e-3)
    # the duration embedding's Linear backward reads its output gradient in bf16 (autocast): the
    # reference rounds each level's token sum to bf16 and sums the levels' four weight gradients, the
    # fused path rounds the sum over all levels once — the same terms, one bf16 rounding apart
    torch.testing.assert_close(w1, w2, rtol=1e-2, atol=1e-2 * w2.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("T,C,G", [(1024, 512, 32), (100, 256, 32), (37, 1024, 16)])
def test_groupnorm_cl_matches_group_norm(dev, T, C, G):
    """pyramid.group_norm_cl (mfl_groupnorm_cl_*): GroupNorm of channels-last bf16 rows written into a
    flattened buffer equals the reference's nn.GroupNorm on the (B, C, T) transpose in fp32 (autocast's
    group_norm), and so do its input / gamma / beta gradients, for a gradient arriving in fp32 rows of
    the buffer plus one through the bf16 copy."""
    pyr = PKG.models.modules.pyramid
    g = torch.Generator(device=dev).manual_seed(21)
    B = 3
    x = (torch.randn(B, T, C, device=dev, generator=g) * 2 + 0.5).bfloat16().requires_grad_(True)
    norm = torch.nn.GroupNorm(G, C).to(dev)
    with torch.no_grad():
        norm.weight.copy_(torch.randn(C, device=dev, generator=g))
        norm.bias.copy_(torch.randn(C, device=dev, generator=g))
    flat = torch.full((B, T + 5, C), float("nan"), device=dev)
    g32 = torch.randn(B, T, C, device=dev, generator=g)
    g16 = torch.randn(B, T, C, device=dev, generator=g).bfloat16()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out32, out16 = pyr.group_norm_cl(x, norm, flat, 5, True)
    ref = torch.nn.functional.group_norm(x.float().transpose(1, 2), G, norm.weight, norm.bias, norm.eps).transpose(1, 2)
    torch.testing.assert_close(out32, ref, rtol=1e-4, atol=1e-4)
    assert torch.equal(out16, out32.bfloat16())
    assert torch.isnan(flat[:, :5]).all() and out32.data_ptr() == flat[:, 5:].data_ptr()
    got = torch.autograd.grad([out32, out16], [x, norm.weight, norm.bias], [g32, g16])
    want = torch.autograd.grad(ref, [x, norm.weight, norm.bias], g32 + g16.float())
    torch.testing.assert_close(got[0].float(), want[0].float(), rtol=2e-2, atol=2e-2 * want[0].abs().max().item())
    torch.testing.assert_close(got[1], want[1], rtol=1e-3, atol=1e-3 * want[1].abs().max().item())
    torch.testing.assert_close(got[2], want[2], rtol=1e-3, atol=1e-3 * want[2].abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("B,T,C", [(2, 64, 256), (8, 1024, 512)])
def test_base_encoder_channels_last_levels_match_reference_path(dev, monkeypatch, B, T, C):
    """BaseEncoder under bf16 autocast with the channels-last GroupNorm (rows written into the flattened
    encoder input, pyramid.flatten_levels joining them without a copy) against the reference's
    composition (MFL_GROUPNORM_CL=0: nn.GroupNorm on the (B, C, T) transposes, torch.cat): every level,
    the flattened input and the input / parameter gradients (reference base_encoder.py:62-89,
    unimodal_deformable_transformer.py:90-134)."""
    torch.manual_seed(5)
    enc = PKG.models.base_encoder.BaseEncoder(4, C, C).to(dev)
    with torch.no_grad():
        for p in enc.parameters():
            p.add_(torch.randn_like(p) * 0.3)
    pos_embed = PKG.models.modules.embedding_layers.PositionEmbeddingVideoSine(C // 2, normalize=True).to(dev)
    video, mask, dur = PKG.dvc_core.synthetic_clips(B, T=T, feature_dim=C, padded=True, seed=3, device=dev)
    video = (video * 1.7 + 0.4).requires_grad_(True)
    pyr = PKG.models.modules.pyramid
    res = []
    for on in ("1", "0"):
        monkeypatch.setenv("MFL_GROUPNORM_CL", on)
        enc.zero_grad(set_to_none=True)
        video.grad = None
        PKG._trace.clear()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            srcs, masks, _ = enc(video, mask, dur, pos_embed)
            flat = pyr.flatten_levels(srcs)
        assert (PKG._trace.hits.get("groupnorm_cl", 0) == 4) == (on == "1"), PKG._trace.hits
        g = torch.randn(flat.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(9))
        (flat * g).sum().backward()
        res.append(([s.detach().float().clone() for s in srcs] + [flat.detach().clone()],
                    [video.grad.clone()] + [p.grad.clone() for p in enc.parameters()]))
    (fa, ga), (fb, gb) = res
    # level 0 as the reference to fp32 summation order; the later levels read the previous level's bf16
    # copy, where an fp32 difference of one ulp can round the other way (the reference rounds its fp32
    # GroupNorm output at the next convolution's cast): held to the norm of the level
    torch.testing.assert_close(fa[0], fb[0], rtol=1e-4, atol=1e-4)
    for i, (a, b) in enumerate(zip(fa, fb)):
        err = ((a.double() - b.double()).norm() / b.double().norm()).item()
        assert err < 1e-3, (i, err)
    for i, (a, b) in enumerate(zip(ga, gb)):
        err = ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()
        assert err < 2e-2, (i, err)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gelu_dropout_matches_aten(dev, p):
    """ffn.gelu_dropout (mfl_gelu_dropout_*): dropout(gelu(h)) of the caption decoder's MLP (reference
    layers.py:827-869, exact erf GELU) with ATen's bf16 roundings — without dropout equal to F.gelu's
    forward and gelu_backward (to one bf16 ulp on a few elements: erf / exp of another math library
    build); with dropout the kept elements are bf16(bf16(gelu) / (1 - p)), about p of them dropped, and
    the backward passes the gradient exactly where the forward kept."""
    ffn = PKG.models.modules.ffn
    g = torch.Generator(device=dev).manual_seed(3)
    h = (torch.randn(3192, 2048, device=dev, generator=g) * 2).bfloat16().requires_grad_(True)
    dy = torch.randn(3192, 2048, device=dev, generator=g).bfloat16()
    drop = torch.nn.Dropout(p).train()
    PKG._trace.clear()
    out = ffn.gelu_dropout(h, torch.nn.GELU(), drop)
    assert PKG._trace.hits.get("gelu_dropout", 0) == 1
    (dx,) = torch.autograd.grad(out, h, dy)
    ref = torch.nn.functional.gelu(h.detach().float()).bfloat16()
    rdx = torch.ops.aten.gelu_backward(dy, h.detach(), approximate="none")

    def ulps(a, b):
        ai = a.view(torch.int16).int()
        bi = b.view(torch.int16).int()
        return (ai - bi).abs()

    if p == 0.0:
        assert (ulps(out, ref) > 1).sum().item() == 0 and (ulps(out, ref) > 0).float().mean().item() < 1e-3
        assert (ulps(dx, rdx) > 1).sum().item() == 0 and (ulps(dx, rdx) > 0).float().mean().item() < 1e-3
    else:
        kept = out != 0
        frac = 1 - kept.float().mean().item()
        assert abs(frac - p) < 0.01, frac
        want = (ref.float() / (1 - p)).bfloat16()
        nz = kept & (ref != 0)
        assert (ulps(out[nz], want[nz]) > 1).sum().item() == 0
        # the backward keeps exactly the forward's elements (where gelu(h) != 0)
        dmask = (dy.float() / (1 - p)).bfloat16()
        want_dx = torch.ops.aten.gelu_backward(dmask, h.detach(), approximate="none")
        assert torch.equal(dx[~kept & (ref != 0)], torch.zeros_like(dx[~kept & (ref != 0)]))
        assert (ulps(dx[nz], want_dx[nz]) > 1).sum().item() == 0


@pytest.mark.gpu
def test_word_probs_fused_backward_matches_dense(dev):
    """unimodal_caption_decoder.word_probs (mfl_word_prob_backward): the caption loss's gather of one
    word's probability a row from the bf16-logit softmax, its gradient written to the logits in one
    pass, equals the dense path's (the gather's scatter into zeros, softmax's backward, the bf16 cast) —
    the same formula c (delta - p) in fp32, one bf16 rounding."""
    ucd = PKG.models.unimodal_caption_decoder
    g = torch.Generator(device=dev).manual_seed(4)
    rows, V = (6, 28, 19), 10000
    x = (torch.randn(*rows, V, device=dev, generator=g) * 3).bfloat16()
    words = torch.randint(0, V, rows, device=dev, generator=g)
    live = (torch.rand(rows, device=dev, generator=g) > 0.2).float()
    res = []
    for fused in (True, False):
        lg = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            probs = ucd._probs(lg)
        assert hasattr(probs, "_mfl_logits")
        p = ucd.word_probs(probs, words) if fused else probs.float().gather(-1, words[..., None])[..., 0]
        loss = -(torch.log(p.clamp_min(1e-9)) * live).sum() / live.sum()
        loss.backward()
        res.append((p.detach(), lg.grad.float()))
    (pa, ga), (pb, gb) = res
    assert torch.equal(pa, pb)
    torch.testing.assert_close(ga, gb, rtol=1e-2, atol=1e-2 * gb.abs().max().item())
    assert ((ga - gb).norm() / gb.norm()).item() < 1e-3
