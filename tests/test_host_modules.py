"""Host logic of the mirrored modules, on CPU, with the MSDA core swapped for the oracle
(oracle.cpu_model.oracle_core): MSDeformAttn, PositionEmbeddingVideoSine + BaseEncoder +
DeformableTransformer and MultimodalDeformableTransformer must reproduce the reference's
golden outputs and gradients (fp64), and the product path must refuse host tensors."""
import pytest
import torch

from conftest import PKG
from oracle.cpu_model import oracle_core

M = PKG.models


def _load(module, sd):
    module.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in sd.items()})
    return module


def _close(a, b, rtol=1e-9, atol=1e-10):
    torch.testing.assert_close(a, b.to(a.dtype), rtol=rtol, atol=atol)


def test_product_core_refuses_cpu_tensors():
    v = torch.zeros(1, 6, 1, 4)
    loc = torch.zeros(1, 2, 1, 2, 1)
    aw = torch.ones(1, 2, 1, 2, 1)
    with pytest.raises(RuntimeError, match="ROCm device"):
        M.modules.attention.ms_deform_attn_core_pytorch(v, torch.tensor([4, 2]), loc, aw)
    with pytest.raises(RuntimeError, match="Not implemented on the CPU"):
        PKG.MultiScaleDeformableAttention.ms_deform_attn_forward(v, torch.tensor([[1, 4], [1, 2]]),
                                                                torch.tensor([0, 4]),
                                                                torch.stack([loc, loc * 0 + 0.5], -1), aw, 64)


def test_host_levels_forms():
    hl = PKG.msda.host_levels
    assert hl(torch.tensor([8, 4, 2])) == ((8, 4, 2), (0, 8, 12))
    assert hl(torch.tensor([[8], [4]])) == ((8, 4), (0, 8))
    assert hl(torch.tensor([[1, 8], [1, 4]]), torch.tensor([0, 8])) == ((8, 4), (0, 8))
    with pytest.raises(NotImplementedError):
        hl(torch.tensor([[2, 8]]))
    t = torch.tensor([5, 3])
    t._mfl_host = (5, 3)
    assert hl(t) == ((5, 3), (0, 5))


@pytest.mark.parametrize("case", ["enc", "enc_masked", "dec"])
def test_msdeformattn_matches_reference(golden, case):
    g = golden("module_f64")
    d = g[case]
    sd = g["state_dict"]
    d_model = sd["value_proj.weight"].shape[0]
    attn = _load(M.modules.attention.MSDeformAttn(d_model, 4, 4, 4).double(), sd)
    shapes = g["shapes"]
    start = torch.cat((shapes.new_zeros(1), shapes.cumsum(0)[:-1]))
    q = d["query"].clone().requires_grad_(True)
    x = d["input_flatten"].clone().requires_grad_(True)
    mask = d["padding_mask"] if d["padding_mask"].numel() else None
    with oracle_core(PKG):
        y, sl, sa = attn(q, d["reference_points"], x, shapes, start, mask, is_sparse=True)
        y.backward(d["grad_out"])
    _close(y, d["output"])
    _close(sl, d["sampling_locations"])
    _close(sa, d["attention_weights"])
    _close(q.grad, d["grad_query"], rtol=1e-8, atol=1e-9)
    _close(x.grad, d["grad_input_flatten"], rtol=1e-8, atol=1e-9)
    for k, p in attn.named_parameters():
        _close(p.grad, d["param_grads"][k], rtol=1e-8, atol=1e-9)


def build_transformer_stack(g, device="cpu"):
    d_model, heads, Q = 64, 4, 20
    pos = M.modules.embedding_layers.PositionEmbeddingVideoSine(d_model // 2, normalize=True)
    base = M.base_encoder.BaseEncoder(4, d_model, d_model)
    tr = M.deformable.unimodal_deformable_transformer.DeformableTransformer(
        d_model=d_model, num_head=heads, num_encoder_layers=2, num_decoder_layers=2, dim_feedforward=128,
        dropout=0.0, return_intermediate_dec=True, num_feature_levels=4, dec_n_points=4, enc_n_points=4)
    qe = torch.nn.Embedding(Q, 2 * d_model)
    mods = {"pos_embed": pos, "base_encoder": base, "transformer": tr, "query_embedding": qe}
    for n, m in mods.items():
        _load(m.double().to(device), g["state_dicts"][n])
    return mods


def run_transformer_stack(mods, video, mask, durations):
    pos, base, tr, qe = (mods[k] for k in ("pos_embed", "base_encoder", "transformer", "query_embedding"))
    B = video.shape[0]
    srcs, masks, poses = base(video, mask, durations, pos)
    src_flatten, shapes, starts, valid, lvl_pos, mask_flatten = tr.prepare_encoder_inputs(srcs, masks, poses)
    memory = tr.forward_encoder(src_flatten, shapes, starts, valid, lvl_pos, mask_flatten)
    qmask = torch.ones(B, qe.weight.shape[0], dtype=torch.bool, device=video.device)
    _, tgt, refp, qpos = tr.prepare_decoder_input_query(B, qe.weight)
    hs, inter = tr.forward_decoder(tgt, refp, memory, shapes, starts, valid, qpos, mask_flatten, qmask, False)
    return memory, hs, inter


def test_transformer_stack_matches_reference(golden):
    g = golden("transformer_f64")
    mods = build_transformer_stack(g)
    video = g["video"].clone().requires_grad_(True)
    torch.set_default_dtype(torch.float64)
    try:
        with oracle_core(PKG):
            memory, hs, inter = run_transformer_stack(mods, video, g["mask"], g["durations"])
            loss = (hs * g["w_hs"]).sum() + (memory * g["w_mem"]).sum()
            loss.backward()
    finally:
        torch.set_default_dtype(torch.float32)
    _close(memory, g["memory"])
    _close(hs, g["hs"])
    _close(inter, g["inter_references"])
    _close(video.grad, g["grad_video"], rtol=1e-8, atol=1e-9)
    for n, m in mods.items():
        for k, p in m.named_parameters():
            if k in g["param_grads"][n]:
                _close(p.grad, g["param_grads"][n][k], rtol=1e-7, atol=1e-9)


def build_multimodal(g, device="cpu"):
    tr = M.deformable.multimodal_deformable_transformer.MultimodalDeformableTransformer(
        d_model=64, num_head=4, num_encoder_layers=1, num_decoder_layers=1, dim_feedforward=128, dropout=0.0,
        return_intermediate_dec=True, num_feature_levels=4, dec_n_points=4, enc_n_points=4)
    qe = torch.nn.Embedding(g["state_dicts"]["query_embedding"]["weight"].shape[0], 128)
    _load(tr.double().to(device), g["state_dicts"]["transformer"])
    _load(qe.double().to(device), g["state_dicts"]["query_embedding"])
    return tr, qe


def run_multimodal(tr, qe, inputs):
    prepared = {n: tr.prepare_encoder_inputs(d["srcs"], d["masks"], d["pos"]) for n, d in inputs.items()}
    v, a = prepared["video"], prepared["audio"]
    mem_v, mem_a = tr.forward_encoder(*v, *a)
    B = mem_v.shape[0]
    qmask = torch.ones(B, qe.weight.shape[0], dtype=torch.bool, device=mem_v.device)
    _, tgt, refp, qpos = tr.prepare_decoder_input_query(B, qe.weight)
    hs, inter = tr.forward_decoder(tgt, refp, qpos, qmask, mem_v, v[1], v[2], v[3], v[5], mem_a, a[1], a[2], a[3],
                                   a[5], False)
    return mem_v, mem_a, hs, inter


def test_multimodal_matches_reference(golden):
    g = golden("multimodal_f64")
    tr, qe = build_multimodal(g)
    inputs = {n: dict(srcs=[s.clone().requires_grad_(True) for s in d["srcs"]], pos=d["pos"], masks=d["masks"])
              for n, d in g["inputs"].items()}
    with oracle_core(PKG):
        mem_v, mem_a, hs, inter = run_multimodal(tr, qe, inputs)
        w = g["weights"]
        ((hs * w[0]).sum() + (mem_v * w[1]).sum() + (mem_a * w[2]).sum()).backward()
    _close(hs, g["hs"])
    _close(mem_v, g["memory_video"])
    _close(mem_a, g["memory_audio"])
    for n in ("video", "audio"):
        for s, ref in zip(inputs[n]["srcs"], g["grad_srcs"][n]):
            _close(s.grad, ref, rtol=1e-8, atol=1e-9)
    for k, p in tr.named_parameters():
        if k in g["param_grads"]["transformer"]:
            _close(p.grad, g["param_grads"]["transformer"][k], rtol=1e-7, atol=1e-9)


def test_cap_module_init_matches_reference_layout(golden):
    """MSDeformAttnCap keeps the reference's 2*d_model query projections and centred offset grid."""
    g = golden("ops_module_f64")
    sd = g["cap"]["state_dict"]
    m = M.ops.modules.MSDeformAttnCap(32, 4, 4, 4)
    assert {k: tuple(v.shape) for k, v in m.state_dict().items()} == {k: tuple(v.shape) for k, v in sd.items()}
    torch.testing.assert_close(m.sampling_offsets.bias, sd["sampling_offsets.bias"].float())


def test_mha_self_attention_matches_module():
    """Decoder query self-attention as one SDPA over the module's parameters (attention.py
    mha_self_attention) equals nn.MultiheadAttention's sequence-first call (reference
    unimodal_deformable_transformer.py:352-353), fp64, with padded queries; gradients too."""
    import torch
    from conftest import PKG
    att = PKG.models.modules.attention
    torch.manual_seed(0)
    mha = torch.nn.MultiheadAttention(64, 8, dropout=0.1).double().eval()
    tgt = torch.randn(3, 10, 64, dtype=torch.float64, requires_grad=True)
    pos = torch.randn(3, 10, 64, dtype=torch.float64)
    qmask = torch.ones(3, 10, dtype=torch.bool)
    qmask[1, 7:] = False
    out = att.mha_self_attention(mha, tgt, pos, qmask)
    qk = (tgt + pos).transpose(0, 1)
    ref = mha(qk, qk, tgt.transpose(0, 1), key_padding_mask=~qmask)[0].transpose(0, 1)
    torch.testing.assert_close(out, ref, rtol=1e-12, atol=1e-12)
    g = torch.randn_like(out)
    ga = torch.autograd.grad(out, [tgt] + list(mha.parameters()), g)
    gb = torch.autograd.grad(ref, [tgt] + list(mha.parameters()), g)
    for a, b in zip(ga, gb):
        torch.testing.assert_close(a, b, rtol=1e-10, atol=1e-10)


def test_segment_memory_crops_compose_and_stack():
    """SegmentMemory (utils/preds_postprocess.py): a crop of a crop is the materialised crop of the
    materialised crop (reference unimodal_deformable_dvc.py:235 rebinds the memory), the
    projection of a crop is the projection of its materialisation (kept rows: the source row's
    projection; zeroed rows: the bias), and ``cat`` stacks crops of one source along the segments."""
    import torch
    from conftest import PKG
    SM = PKG.utils.preds_postprocess.SegmentMemory
    g = torch.Generator().manual_seed(4)
    B, K, d = 3, 40, 16
    src = torch.randn(B, K, d, generator=g, dtype=torch.float64)
    m0 = SM.of(src)
    bid1 = torch.tensor([0, 2, 2, 1])
    keep1 = torch.rand(4, K, generator=g) < 0.6
    m1 = m0.select(bid1, keep1)
    ref1 = torch.where(keep1[..., None], src[bid1], 0.0)
    assert torch.equal(m1.materialize(), ref1)
    bid2 = torch.tensor([1, 0, 3, 3, 2])
    keep2 = torch.rand(5, K, generator=g) < 0.7
    m2 = m1.select(bid2, keep2)
    assert torch.equal(m2.materialize(), torch.where(keep2[..., None], ref1[bid2], 0.0))
    lin = torch.nn.Linear(d, d).double()
    assert torch.allclose(m2.project(lin), lin(m2.materialize()), rtol=0, atol=1e-12)
    both = SM.cat([m1, m2])
    assert torch.equal(both.materialize(), torch.cat([m1.materialize(), m2.materialize()]))
    assert both.cache is m1.cache


@pytest.mark.parametrize("k,T", [(1, 16), (3, 16), (3, 15)])
def test_conv1d_as_gemm_equals_conv1d(k, T):
    """The BaseEncoder's Conv1d lowering (models/base_encoder.py _Conv1dGemm: the taps' shifted
    channels-last rows side by side, one GEMM; the input gradient folded back) computes
    F.conv1d and its gradients exactly in fp64 (k=1, and k=3 stride 2 padding 1 with even / odd T;
    reference base_encoder.py:27-36)."""
    import importlib
    be = importlib.import_module(PKG.__name__ + ".models.base_encoder")
    torch.manual_seed(0)
    conv = torch.nn.Conv1d(8, 6, kernel_size=k, stride=1 if k == 1 else 2, padding=0 if k == 1 else 1).double()
    x = torch.randn(2, T, 8, dtype=torch.float64, requires_grad=True)
    y = be._Conv1dGemm.apply(x, conv.weight, conv.bias)
    g = torch.randn_like(y)
    got = (y,) + torch.autograd.grad(y, (x, conv.weight, conv.bias), g)
    x2 = x.detach().clone().requires_grad_(True)
    y2 = conv(x2.transpose(1, 2)).transpose(1, 2)
    want = (y2,) + torch.autograd.grad(y2, (x2, conv.weight, conv.bias), g)
    for a, b in zip(got, want):
        torch.testing.assert_close(a, b, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("dur_dtype", [torch.float32, torch.float64])
def test_crop_masks_of_all_levels_equal_the_level_loop(dur_dtype):
    """preds_postprocess.crop_segments builds every pyramid level's token range at once; it equals the
    reference's loop over the levels (crop_segments :481-490: per level, start / end =
    clamp(round(lower + diff * t / duration)), the union of the ranges) element for element, with
    float32 and float64 durations (the arithmetic promotes the same way)."""
    pp = PKG.utils.preds_postprocess
    g = torch.Generator().manual_seed(2)
    B, n, K, L, R = 8, 60, 1920, 4, 1024
    durs = torch.rand(B, generator=g, dtype=dur_dtype) * 230 + 10
    bid = torch.randint(0, B, (n,), generator=g)
    seg = torch.sort(torch.rand(n, 2, generator=g) * durs[bid][:, None].float() * 1.1, 1)[0]
    seg[:3] = torch.tensor([[0.0, 0.0], [5.0, 5.0], [0.0, 1e4]])  # empty, point, past the end
    dur = pp._durations(durs, seg.device)[bid]
    tok = torch.arange(K)
    want = torch.zeros(n, K, dtype=torch.bool)
    for lower, upper in pp.level_token_ranges(L, R):
        diff = upper - lower
        s = torch.clamp((lower + (diff * seg[:, 0] / dur)).round().long(), min=lower, max=upper - 1)
        e = torch.clamp((lower + (diff * seg[:, 1] / dur)).round().long(), min=lower, max=upper - 1)
        want |= (tok[None, :] >= s[:, None]) & (tok[None, :] < e[:, None])
    _, key_mask = pp.crop_segments(torch.zeros(B, K, 4), seg, bid, durs, L, R)
    assert torch.equal(~key_mask, want)
