"""Generate the golden vectors under tests/golden/ by running the REAL reference on CPU.

Run in the build container (where /root/reference exists):
    PYTHONDONTWRITEBYTECODE=1 python3 -B tests/golden/make_golden.py

The reference is imported read-only from /root/reference (no bytecode written there),
with stub modules for packages it imports but never uses on this path (torchvision,
torchaudio, timm, wandb, ml_collections) and a namespace shim for ``models`` that skips
``models/__init__.py`` (which imports timm).  Only tensors are written (torch.save of a
dict of tensors, loadable with ``weights_only=True``); no reference source is copied.

Fixtures:
  op_border_{f64,f32}.pt     ms_deform_attn_core_pytorch (attention.py:331) fwd + grads,
                             small shapes, locations in U(-0.2, 1.2) + exact border /
                             integer-position points.
  op_border_f32_enc.pt       same at the T=1024 encoder level shapes [1024,512,256,128]
                             (B=1, M=8, D=64, 48 queries); inputs regenerated from a seed,
                             grad_value stored as per-row channel sums + 256 full rows.
  module_f64.pt              MSDeformAttn(d=64, L=4, M=4, P=4) (attention.py:394) fwd + grads,
                             encoder shape (+ padding mask) and decoder shape, is_sparse outputs.
  transformer_f64.pt         PositionEmbeddingVideoSine + BaseEncoder + DeformableTransformer
                             (2 enc + 2 dec, d=64, dropout 0) at T=64, B=2 (one padded clip),
                             sampling_offsets weights jittered off their exact init.
  multimodal_f64.pt          MultimodalDeformableTransformer (1 enc + 1 dec, d=64), video
                             T=32 / audio T=16 pyramids, B=2, offsets jittered likewise.
  dam_f32.pt                 utils/dam.py attn_map_to_flat_grid / idx_to_flat_grid / compute_corr
                             (Sparse-DETR decoder attention map), B=2, 3 layers, M=4, [32,16,8,4],
                             locations in U(-0.2, 1.2) plus integer / border points.
  sparse_f64.pt              SparseDeformableTransformer (rho=0.3: mask predictor, top-k encoder
                             queries scattered back; 2 enc + 2 dec, d=64) fwd + grads, with the
                             decoder attention map of its own sampling locations.
  ops_api_f64.pt             the extension-API 2-D form: ops/functions/ms_deform_attn_func.py:44-71 on
                             (L,2) [H=1, W] shapes with (...,2) [x, y] locations, border as written and
                             with zero padding (the extension kernel's; see _zeros_padding), y-grads;
                             return_value stacks of that core and of attention.py:376-378.
  ops_module_f64.pt          ops/modules MSDeformAttn (through the zero-padding kernel, as on a GPU) and
                             MSDeformAttnCap (border, return_value), enc / dec, padding mask.
  transformer_bf16.pt        transformer_f64's model and inputs under torch.autocast('cpu', bfloat16).
  sparse_dvc_f64.pt          UnimodalSparseDVC end to end as written (train fwd + grads, greedy decode).
  deformable_dvc_f64.pt      UnimodalDeformableDVC with its caption-decoder call's argument order fixed.
  mm_caption_decoder_f64.pt  MultimodalCaptionDecoder with HEAD's undefined names bound (no file edits).
  mm_dvc_f64.pt              MultimodalDeformableDVC training fwd + grads, undefined names bound likewise.
  transformer_bf16_d256.pt   BaseEncoder + DeformableTransformer (2 enc + 2 dec) at d=256, 8 heads, ff 1024,
                             T=64, B=2 (one padded clip), dropout 0: the reference's fp64 run and its run
                             under torch.autocast('cpu', bfloat16) — d % 256 == 0, so the GPU test runs the
                             bench's fused composition on it.  Parameters regenerated from their names
                             (regen_parameters, no state_dict stored); gradients stored on fixed index
                             samples (grad_sample_index) plus their full norms.
  caption_bf16.pt            UnimodalCaptionDecoder at d=512, 8 heads, depth 2, vocab 10000, seq_len 20:
                             teacher-forced forward + gradients of -sum p(target word) and the reference's
                             greedy re-decode loop (unimodal_deformable_dvc.py:304-354), fp64 and bf16 autocast.
  sparse_bf16_d256.pt        BaseEncoder + SparseDeformableTransformer (rho 0.3, 2 enc + 2 dec, d=256, 4 heads
                             of 64, ff 1024), T=64, B=2 (one padded clip), dropout 0: fp64 and bf16 autocast,
                             the seed chosen so that both runs select the same top-k tokens with a margin;
                             outputs, mask prediction, top-k, sampled gradients.
  multimodal_bf16_d256.pt    shared BaseEncoder + MultimodalDeformableTransformer (2 enc + 2 dec, d=256, 4 heads
                             of 64, ff 1024), video T=64 + audio T=16, B=2 (one padded clip), dropout 0: fp64 and
                             bf16 autocast; both memories, hs, input gradients, sampled parameter gradients.

usage: make_golden.py [case ...]   (default: every case; e.g. ``make_golden.py dam sparse``)
"""
import math
import os
import sys
import types

import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True


def _stub(name, **attrs):
    mod = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(mod, k, v)
    sys.modules[name] = mod
    return mod


def import_reference():
    for name in ("torchvision", "torchaudio", "timm", "wandb", "ml_collections"):
        _stub(name, __version__="0.0.0")
    _stub("torchaudio.compliance")
    _stub("torchaudio.compliance.kaldi")
    models = types.ModuleType("models")
    models.__path__ = [os.path.join(REF, "models")]
    sys.modules["models"] = models
    sys.path.insert(0, REF)
    import models.modules.attention as attention  # noqa: E402
    import models.base_encoder as base_encoder  # noqa: E402
    import models.modules.embedding_layers as embedding_layers  # noqa: E402
    import models.deformable.unimodal_deformable_transformer as uni  # noqa: E402
    import models.deformable.multimodal_deformable_transformer as mm  # noqa: E402
    import models.sparse.unimodal_sparse_deformable_transformer as sparse  # noqa: E402
    import importlib.util
    spec = importlib.util.spec_from_file_location("_ref_dam", os.path.join(REF, "utils", "dam.py"))
    dam = importlib.util.module_from_spec(spec)  # utils/dam.py alone: numpy + torch only
    spec.loader.exec_module(dam)
    return types.SimpleNamespace(attention=attention, base_encoder=base_encoder,
                                 embedding_layers=embedding_layers, uni=uni, mm=mm, sparse=sparse, dam=dam)


def _jitter_offsets(module, seed):
    """Move every MSDeformAttn off its exact initialisation: at init all sampling offsets are
    integers, so every encoder sample sits exactly on a map position, where the location
    gradient is discontinuous and any rounding difference picks another segment.  A small
    random sampling_offsets weight (as after a few training steps) puts samples at generic
    positions, so fp32 vs fp64 comparisons of the transformer gradients are meaningful."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for mod in module.modules():
            if type(mod).__name__ == "MSDeformAttn":
                w = mod.sampling_offsets.weight
                w.copy_((torch.randn(w.shape, generator=g, dtype=torch.float64) * 0.05).to(w.dtype))


def _compact(state_dict):
    """fp64 copies of fp32-initialised weights are exactly fp32: store them as fp32."""
    out = {}
    for k, v in state_dict.items():
        if v.dtype == torch.float64 and torch.equal(v.float().double(), v):
            v = v.float()
        out[k] = v.clone()
    return out


def _locations(gen, shape, dtype):
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 1.4 - 0.2).to(dtype)


def _attn(gen, shape, dtype):
    a = torch.rand(shape, generator=gen, dtype=torch.float64) + 1e-5
    a = a / a.sum(-1, keepdim=True).sum(-2, keepdim=True)
    return a.to(dtype)


def _edge_points(loc, shapes):
    """Exact border / integer-position locations for query 0 (binary fractions: exact in fp32)."""
    for l, T in enumerate(shapes):
        pts = [0.5 / T, (T - 0.5) / T, 5.5 / T if T > 6 else 1.5 / T, 0.0, 1.0, -0.5, 1.5]
        flat = loc[:, 0, :, l].reshape(-1)
        for i, v in enumerate(pts):
            if i < flat.numel():
                flat[i] = v
        loc[:, 0, :, l] = flat.view(loc[:, 0, :, l].shape)
    return loc


def _name_seed(name, seed):
    import zlib
    return (zlib.crc32(name.encode()) ^ (seed * 2654435761)) & 0x7FFFFFFF


KEEP_INIT = ("sampling_offsets.bias",)  # the reference's deterministic offset grid (attention.py:427-435)


def regen_parameters(module, seed, scale=None):
    """Overwrite every parameter of ``module`` with values that depend only on its state_dict name
    and ``seed`` (construction-order free), so a fixture stores no weights: the GPU test rebuilds
    the same values on the mirrored modules, whose parameter names are the reference's.
    LayerNorm / GroupNorm weights 1 + U(-0.1, 0.1); other vectors U(-0.05, 0.05); matrices and
    convolutions xavier-uniform bounds; embeddings and ``level_embed`` N(0, 1);
    ``sampling_offsets.weight`` N(0, 0.05) (generic sample positions, as _jitter_offsets);
    ``scale`` multiplies named parameters afterwards.  Returns {name: sum of |p|} (checked by the test)."""
    kinds = {}
    for mname, mod in module.named_modules():
        for pname, _ in mod.named_parameters(recurse=False):
            full = f"{mname}.{pname}" if mname else pname
            if isinstance(mod, (torch.nn.LayerNorm, torch.nn.GroupNorm)):
                kinds[full] = "norm_" + pname
            elif isinstance(mod, torch.nn.Embedding) or pname == "level_embed":
                kinds[full] = "embedding"
            else:
                kinds[full] = "other"
    sums = {}
    with torch.no_grad():
        for name, p in sorted(module.named_parameters()):
            if name.endswith(KEEP_INIT):
                sums[name] = p.double().abs().sum().item()
                continue
            g = torch.Generator().manual_seed(_name_seed(name, seed))
            u = torch.rand(p.shape, generator=g, dtype=torch.float64) * 2 - 1
            kind = kinds[name]
            if kind == "embedding":
                v = torch.randn(p.shape, generator=g, dtype=torch.float64)
            elif kind == "norm_weight":
                v = 1 + 0.1 * u
            elif name.endswith("sampling_offsets.weight"):
                v = torch.randn(p.shape, generator=g, dtype=torch.float64) * 0.05
            elif p.dim() >= 2:
                rf = 1
                for k in p.shape[2:]:
                    rf *= k
                v = u * (6.0 / (p.shape[0] * rf + p.shape[1] * rf)) ** 0.5
            else:
                v = 0.05 * u
            if scale and name in scale:
                v = v * scale[name]
            p.copy_(v.to(p.dtype))
            sums[name] = p.double().abs().sum().item()
    return sums


def grad_sample_index(name, n, k=2048):
    """Fixed sample of a flattened gradient's positions (all of them when n <= k)."""
    if n <= k:
        return torch.arange(n)
    g = torch.Generator().manual_seed(_name_seed(name, 7))
    return torch.randperm(n, generator=g)[:k].sort().values


def sampled_grads(named):
    """{module: {param: (sample of the flat gradient (fp32), full norm (fp64))}}"""
    out = {}
    for mname, m in named.items():
        d = {}
        for k, p in m.named_parameters():
            if p.grad is None:
                continue
            flat = p.grad.reshape(-1)
            d[k] = dict(sample=flat[grad_sample_index(mname + "." + k, flat.numel())].float(),
                        norm=torch.tensor(flat.double().norm().item(), dtype=torch.float64))
        out[mname] = d
    return out


def op_case(ref, dtype, shapes, B, M, D, Lq, P, seed, edge=True):
    gen = torch.Generator().manual_seed(seed)
    L, S = len(shapes), sum(shapes)
    value = torch.randn((B, S, M, D), generator=gen, dtype=torch.float64).to(dtype)
    loc = _locations(gen, (B, Lq, M, L, P), dtype)
    if edge:
        loc = _edge_points(loc, shapes)
    aw = _attn(gen, (B, Lq, M, L, P), dtype)
    gout = torch.randn((B, Lq, M * D), generator=gen, dtype=torch.float64).to(dtype)
    v, lc, a = (t.clone().requires_grad_(True) for t in (value, loc, aw))
    shp = torch.tensor(shapes, dtype=torch.long).unsqueeze(-1)
    out = ref.attention.ms_deform_attn_core_pytorch(v, shp, lc.unsqueeze(-1), a)
    out.backward(gout)
    return dict(value=value, loc=loc, aw=aw, grad_out=gout, shapes=torch.tensor(shapes), out=out.detach(),
                grad_value=v.grad, grad_loc=lc.grad, grad_aw=a.grad)


def op_enc_case(ref, seed=7):
    shapes, B, M, D, Lq, P = [1024, 512, 256, 128], 1, 8, 64, 48, 4
    d = op_case(ref, torch.float32, shapes, B, M, D, Lq, P, seed, edge=True)
    gv = d.pop("grad_value")
    rows = torch.randperm(sum(shapes), generator=torch.Generator().manual_seed(seed + 1))[:256]
    # keep only rows that matter + make the inputs regenerable from the seed
    for k in ("value", "loc", "aw", "grad_out"):
        d.pop(k)
    d.update(seed=torch.tensor(seed), B=torch.tensor(B), M=torch.tensor(M), D=torch.tensor(D),
             Lq=torch.tensor(Lq), P=torch.tensor(P), grad_value_rowsum=gv.sum(-1),
             grad_value_rows=rows, grad_value_at_rows=gv[:, rows])
    return d


def module_case(ref, seed=11):
    torch.manual_seed(seed)
    d_model, L, M, P, B = 64, 4, 4, 4, 2
    shapes = [32, 16, 8, 4]
    S = sum(shapes)
    attn = ref.attention.MSDeformAttn(d_model, L, M, P).double()
    gen = torch.Generator().manual_seed(seed)
    out = {"state_dict": _compact(attn.state_dict()), "shapes": torch.tensor(shapes)}
    shp = torch.tensor(shapes, dtype=torch.long)
    start = torch.cat((shp.new_zeros(1), shp.cumsum(0)[:-1]))
    valid = torch.ones(B, 4)
    valid[1] = torch.tensor([0.75, 0.75, 0.75, 0.75])
    mask = torch.zeros(B, S, dtype=torch.bool)
    for l, (T, s0) in enumerate(zip(shapes, start.tolist())):
        mask[1, s0 + int(T * 0.75):s0 + T] = True
    enc_ref = ref.uni.DeformableTransformerEncoder.get_reference_points(shp, valid.double(), "cpu")
    cases = {
        "enc": (S, enc_ref, None),
        "enc_masked": (S, enc_ref, mask),
        "dec": (20, torch.rand((B, 20, 1), generator=gen, dtype=torch.float64)[:, :, None] * valid.double()[:, None, :, None], None),
    }
    flat0 = torch.randn((B, S, d_model), generator=gen, dtype=torch.float64)
    for name, (Lq, refp, m) in cases.items():
        query = torch.randn((B, Lq, d_model), generator=gen, dtype=torch.float64).requires_grad_(True)
        flat = flat0.clone().requires_grad_(True)
        gout = torch.randn((B, Lq, d_model), generator=gen, dtype=torch.float64)
        attn.zero_grad()
        y, sl, sa = attn(query, refp, flat, shp, start, m, is_sparse=True)
        y.backward(gout)
        out[name] = dict(query=query.detach(), reference_points=refp, input_flatten=flat.detach(),
                         padding_mask=(m if m is not None else torch.zeros(0, dtype=torch.bool)),
                         grad_out=gout, output=y.detach(), sampling_locations=sl.detach(),
                         attention_weights=sa.detach(), grad_query=query.grad, grad_input_flatten=flat.grad,
                         param_grads={k: p.grad.clone() for k, p in attn.named_parameters()})
    return out


def transformer_case(ref, seed=23):
    torch.manual_seed(seed)
    d_model, heads, Q = 64, 4, 20
    pos_embed = ref.embedding_layers.PositionEmbeddingVideoSine(d_model // 2, normalize=True).double()
    base = ref.base_encoder.BaseEncoder(4, d_model, d_model).double()
    tr = ref.uni.DeformableTransformer(d_model=d_model, num_head=heads, num_encoder_layers=2, num_decoder_layers=2,
                                       dim_feedforward=128, dropout=0.0, return_intermediate_dec=True,
                                       num_feature_levels=4, dec_n_points=4, enc_n_points=4).double()
    query_embedding = torch.nn.Embedding(Q, d_model * 2).double()
    _jitter_offsets(tr, seed)
    # the reference's duration embedding allocates with the default dtype
    # (embedding_layers.py:222): run the forward with float64 as the default dtype
    torch.set_default_dtype(torch.float64)
    try:
        return _transformer_run(ref, seed, pos_embed, base, tr, query_embedding)
    finally:
        torch.set_default_dtype(torch.float32)


def _transformer_run(ref, seed, pos_embed, base, tr, query_embedding):
    d_model, B, T, Q = 64, 2, 64, 20
    gen = torch.Generator().manual_seed(seed)
    video = torch.randn((B, T, d_model), generator=gen, dtype=torch.float64).requires_grad_(True)
    mask = torch.zeros(B, T, dtype=torch.bool)
    mask[1, 48:] = True
    durations = torch.tensor([37.5, 120.2], dtype=torch.float64)
    srcs, masks, pos = base(video, mask, durations, pos_embed)
    src_flatten, shapes, starts, valid, lvl_pos, mask_flatten = tr.prepare_encoder_inputs(srcs, masks, pos)
    memory = tr.forward_encoder(src_flatten, shapes, starts, valid, lvl_pos, mask_flatten)
    qmask = torch.ones(B, Q, dtype=torch.bool)
    init_ref, tgt, refp, qe = tr.prepare_decoder_input_query(B, query_embedding.weight)
    hs, inter = tr.forward_decoder(tgt, refp, memory, shapes, starts, valid, qe, mask_flatten, qmask, False)
    w_hs = torch.randn(hs.shape, generator=gen, dtype=torch.float64)
    w_mem = torch.randn(memory.shape, generator=gen, dtype=torch.float64)
    loss = (hs * w_hs).sum() + (memory * w_mem).sum()
    loss.backward()
    named = {"pos_embed": pos_embed, "base_encoder": base, "transformer": tr, "query_embedding": query_embedding}
    return dict(
        video=video.detach(), mask=mask, durations=durations, w_hs=w_hs, w_mem=w_mem,
        memory=memory.detach(), hs=hs.detach(), inter_references=inter.detach(), loss=loss.detach(),
        grad_video=video.grad,
        state_dicts={n: _compact(m.state_dict()) for n, m in named.items()},
        param_grads={n: {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
                     for n, m in named.items()})


def multimodal_case(ref, seed=31):
    torch.manual_seed(seed)
    d_model, heads, B, Q = 64, 4, 2, 12
    tr = ref.mm.MultimodalDeformableTransformer(d_model=d_model, num_head=heads, num_encoder_layers=1,
                                                num_decoder_layers=1, dim_feedforward=128, dropout=0.0,
                                                return_intermediate_dec=True, num_feature_levels=4,
                                                dec_n_points=4, enc_n_points=4).double()
    query_embedding = torch.nn.Embedding(Q, d_model * 2).double()
    _jitter_offsets(tr, seed)
    gen = torch.Generator().manual_seed(seed)
    inputs = {}
    prepared = {}
    for name, lens in (("video", [32, 16, 8, 4]), ("audio", [16, 8, 4, 2])):
        srcs = [torch.randn((B, d_model, t), generator=gen, dtype=torch.float64).requires_grad_(True) for t in lens]
        pos = [torch.randn((B, d_model, t), generator=gen, dtype=torch.float64) for t in lens]
        masks = [torch.zeros(B, t, dtype=torch.bool) for t in lens]
        masks = [m.clone() for m in masks]
        for m, t in zip(masks, lens):
            m[1, (3 * t) // 4:] = True
        inputs[name] = dict(srcs=srcs, pos=pos, masks=masks)
        prepared[name] = tr.prepare_encoder_inputs(srcs, masks, pos)
    v, a = prepared["video"], prepared["audio"]
    mem_v, mem_a = tr.forward_encoder(*v, *a)
    qmask = torch.ones(B, Q, dtype=torch.bool)
    init_ref, tgt, refp, qe = tr.prepare_decoder_input_query(B, query_embedding.weight)
    hs, inter = tr.forward_decoder(tgt, refp, qe, qmask, mem_v, v[1], v[2], v[3], v[5], mem_a, a[1], a[2], a[3], a[5],
                                   False)
    w = [torch.randn(t.shape, generator=gen, dtype=torch.float64) for t in (hs, mem_v, mem_a)]
    loss = (hs * w[0]).sum() + (mem_v * w[1]).sum() + (mem_a * w[2]).sum()
    loss.backward()
    return dict(
        inputs={n: dict(srcs=[s.detach() for s in d["srcs"]], pos=d["pos"], masks=d["masks"]) for n, d in inputs.items()},
        grad_srcs={n: [s.grad for s in d["srcs"]] for n, d in inputs.items()},
        weights=w, hs=hs.detach(), inter_references=inter.detach(), memory_video=mem_v.detach(),
        memory_audio=mem_a.detach(), loss=loss.detach(),
        state_dicts={"transformer": _compact(tr.state_dict()), "query_embedding": _compact(query_embedding.state_dict())},
        param_grads={"transformer": {k: p.grad.clone() for k, p in tr.named_parameters() if p.grad is not None},
                     "query_embedding": {k: p.grad.clone() for k, p in query_embedding.named_parameters()}})


def dam_case(ref, seed=41):
    gen = torch.Generator().manual_seed(seed)
    shapes, B, NL, Lq, M, P = [32, 16, 8, 4], 2, 3, 20, 4, 4
    L = len(shapes)
    loc = _locations(gen, (B, NL, Lq, M, L, P), torch.float32)
    for l, T in enumerate(shapes):  # integer and border positions (loc * T exact in fp32)
        loc[0, 0, 0, :, l, :] = torch.tensor([0.0, 1.0 / T, (T - 1.0) / T, 1.0]).view(1, 4).expand(M, 4)
    aw = torch.rand((B, NL, Lq, M, L, P), generator=gen, dtype=torch.float32)
    shp = torch.tensor(shapes, dtype=torch.long)
    start = torch.cat((shp.new_zeros(1), shp.cumsum(0)[:-1]))
    grid = ref.dam.attn_map_to_flat_grid(shp, start, loc.unsqueeze(-1), aw)
    summed = grid.sum(dim=(1, 2))
    topk = torch.topk(summed, 10)[1]
    flat_topk = ref.dam.idx_to_flat_grid(shp, topk)
    corr = ref.dam.compute_corr(flat_topk, summed, shp)
    return dict(shapes=shp, level_start=start, loc=loc, aw=aw, flat_grid=grid, topk=topk, flat_topk=flat_topk,
                corr=torch.stack(corr))


def sparse_case(ref, seed=53):
    torch.manual_seed(seed)
    d_model, heads, B, Q = 64, 4, 2, 12
    tr = ref.sparse.SparseDeformableTransformer(d_model=d_model, num_head=heads, num_encoder_layers=2,
                                                num_decoder_layers=2, dim_feedforward=128, dropout=0.0,
                                                return_intermediate_dec=True, num_feature_levels=4,
                                                dec_n_points=4, enc_n_points=4, rho=0.3).double()
    query_embedding = torch.nn.Embedding(Q, d_model * 2).double()
    _jitter_offsets(tr, seed)
    gen = torch.Generator().manual_seed(seed)
    lens = [32, 16, 8, 4]
    srcs = [torch.randn((B, d_model, t), generator=gen, dtype=torch.float64).requires_grad_(True) for t in lens]
    pos = [torch.randn((B, d_model, t), generator=gen, dtype=torch.float64) for t in lens]
    masks = [torch.zeros(B, t, dtype=torch.bool) for t in lens]
    for m, t in zip(masks, lens):
        m[1, (3 * t) // 4:] = True
    (src_flatten, shapes, starts, valid, lvl_pos, mask_flatten, proposals, topk, mask_pred,
     sparse_token_nums) = tr.prepare_encoder_inputs(srcs, masks, pos)
    memory, sl_enc, aw_enc, _, _ = tr.forward_encoder(src_flatten, shapes, starts, valid, lvl_pos, mask_flatten,
                                                      proposals, topk, sparse_token_nums)
    qmask = torch.ones(B, Q, dtype=torch.bool)
    init_ref, tgt, refp, qe = tr.prepare_decoder_input_query(B, query_embedding.weight)
    hs, inter, sl_dec, aw_dec = tr.forward_decoder(tgt, refp, memory, shapes, starts, valid, qe, mask_flatten, qmask,
                                                   False)
    dam = ref.dam.attn_map_to_flat_grid(shapes, starts, sl_dec.detach().float(), aw_dec.detach().float())
    w = [torch.randn(t.shape, generator=gen, dtype=torch.float64) for t in (hs, memory, mask_pred)]
    loss = (hs * w[0]).sum() + (memory * w[1]).sum() + (mask_pred * w[2]).sum()
    loss.backward()
    return dict(
        srcs=[s.detach() for s in srcs], pos=pos, masks=masks, weights=w, hs=hs.detach(), memory=memory.detach(),
        mask_prediction=mask_pred.detach(), topk=topk, sparse_token_nums=sparse_token_nums,
        sampling_locations_enc=sl_enc.detach(), attn_weights_enc=aw_enc.detach(),
        sampling_locations_dec=sl_dec.detach(), attn_weights_dec=aw_dec.detach(), dam_flat_grid=dam,
        grad_srcs=[s.grad for s in srcs], loss=loss.detach(),
        state_dicts={"transformer": _compact(tr.state_dict()), "query_embedding": _compact(query_embedding.state_dict())},
        param_grads={"transformer": {k: p.grad.clone() for k, p in tr.named_parameters() if p.grad is not None},
                     "query_embedding": {k: p.grad.clone() for k, p in query_embedding.named_parameters()}})


class _zeros_padding:
    """Inside the reference's ops core (models/ops/functions/ms_deform_attn_func.py:61-62) force
    ``F.grid_sample``'s padding to 'zeros': the padding of the extension kernel that the reference's
    own test compares this core against (models/ops/test.py:38-39; ms_deform_im2col_cuda.cuh:34-85).
    Only the module attribute ``F`` of the imported module object is swapped, for the duration."""

    def __init__(self, ref):
        self.mod = ref.ops_func

    def __enter__(self):
        real = torch.nn.functional

        def grid_sample(*args, **kw):
            kw["padding_mode"] = "zeros"
            return real.grid_sample(*args, **kw)

        self.saved = self.mod.F
        self.mod.F = types.SimpleNamespace(grid_sample=grid_sample)
        return self

    def __exit__(self, *exc):
        self.mod.F = self.saved
        return False


def _import_ops(ref):
    import models.ops.functions.ms_deform_attn_func as ops_func  # noqa: E402 (extension import is try/except)
    import models.ops.modules.ms_deform_attn as ops_mod  # noqa: E402
    import models.ops.modules.ms_deform_attn_for_caption as ops_cap  # noqa: E402
    ref.ops_func, ref.ops_mod, ref.ops_cap = ops_func, ops_mod, ops_cap
    return ref


def ops_api_case(ref, seed=61):
    """The extension-API forms: the reference's 2-D core
    (ops/functions/ms_deform_attn_func.py:44-71) on (L,2) [H=1, W=T] shapes with (...,2) [x, y]
    locations — border as written, and zeros (the extension kernel's padding, see _zeros_padding) —
    with all gradients including y; the ``return_value`` stacks of both cores (ops :67-68 and the
    live attention.py:376-378) with the gradients of a weighted sum of the stack."""
    _import_ops(ref)
    gen = torch.Generator().manual_seed(seed)
    shapes, B, M, D, Lq, P = [32, 16, 8, 4], 2, 4, 8, 20, 4
    L, S = len(shapes), sum(shapes)
    value = torch.randn((B, S, M, D), generator=gen, dtype=torch.float64)
    x = _edge_points(_locations(gen, (B, Lq, M, L, P), torch.float64), shapes)
    y = torch.rand((B, Lq, M, L, P), generator=gen, dtype=torch.float64) * 2.2 - 0.6  # row weight live in (-0.5, 1.5)
    loc2 = torch.stack([x, y], -1)
    aw = _attn(gen, (B, Lq, M, L, P), torch.float64)
    gout = torch.randn((B, Lq, M * D), generator=gen, dtype=torch.float64)
    shp2 = torch.tensor([[1, t] for t in shapes], dtype=torch.long)
    out = dict(value=value, loc2=loc2, aw=aw, grad_out=gout, shapes2d=shp2)
    for mode in ("border", "zeros"):
        v, lc, a = (t.clone().requires_grad_(True) for t in (value, loc2, aw))
        if mode == "zeros":
            with _zeros_padding(ref):
                o = ref.ops_func.ms_deform_attn_core_pytorch(v, shp2, lc, a)
        else:
            o = ref.ops_func.ms_deform_attn_core_pytorch(v, shp2, lc, a)
        o.backward(gout)
        out[mode] = dict(out=o.detach(), grad_value=v.grad, grad_loc=lc.grad, grad_aw=a.grad)
    # return_value stacks: (B*M, D, Lq, L, P)
    w_stack = torch.randn((B * M, D, Lq, L, P), generator=gen, dtype=torch.float64)
    out["w_stack"] = w_stack
    for name in ("ops_border", "ops_zeros", "live"):
        v, lc, a = (t.clone().requires_grad_(True) for t in (value, loc2, aw))
        if name == "live":
            st = ref.attention.ms_deform_attn_core_pytorch(v, torch.tensor(shapes).unsqueeze(-1), lc[..., :1], a,
                                                           return_value=True)
        elif name == "ops_zeros":
            with _zeros_padding(ref):
                st = ref.ops_func.ms_deform_attn_core_pytorch(v, shp2, lc, a, return_value=True)
        else:
            st = ref.ops_func.ms_deform_attn_core_pytorch(v, shp2, lc, a, return_value=True)
        (st * w_stack).sum().backward()
        out["stack_" + name] = dict(stack=st.detach(), grad_value=v.grad, grad_loc=lc.grad)
    return out


def ops_module_case(ref, seed=67):
    """The extension-backed modules: ops/modules/ms_deform_attn.py ``MSDeformAttn`` (1-D -> 2-D lift,
    zero-init attention weights) as it runs on a GPU, i.e. through the zero-padding kernel
    (:119-122; reproduced by _zeros_padding on the CPU core), and ``MSDeformAttnCap``
    (ms_deform_attn_for_caption.py: 2*d_model queries, border core with return_value).
    Attention-weight and offset weights are randomised so the softmax and locations are generic."""
    _import_ops(ref)
    torch.manual_seed(seed)
    d_model, L, M, P, B = 32, 4, 4, 4, 2
    shapes = [32, 16, 8, 4]
    S = sum(shapes)
    gen = torch.Generator().manual_seed(seed)
    shp = torch.tensor(shapes, dtype=torch.long)
    start = torch.cat((shp.new_zeros(1), shp.cumsum(0)[:-1]))
    mask = torch.zeros(B, S, dtype=torch.bool)
    for T, s0 in zip(shapes, start.tolist()):
        mask[1, s0 + (3 * T) // 4:s0 + T] = True
    res = {"shapes": shp}
    for name, cls, qdim in (("attn", ref.ops_mod.MSDeformAttn, d_model), ("cap", ref.ops_cap.MSDeformAttnCap,
                                                                          2 * d_model)):
        m = cls(d_model, L, M, P).double()
        with torch.no_grad():
            for lin in (m.sampling_offsets, m.attention_weights):
                lin.weight.copy_(torch.randn(lin.weight.shape, generator=gen, dtype=torch.float64) * 0.05)
        entry = {"state_dict": _compact(m.state_dict())}
        for case, Lq, refdim in (("enc", S, 1), ("dec", 12, 2)):
            if refdim == 1:
                refp = torch.rand((B, Lq, 1), generator=gen, dtype=torch.float64)[:, :, None].expand(B, Lq, L, 1)
            else:
                c = torch.rand((B, Lq, 1), generator=gen, dtype=torch.float64) * 0.8 + 0.1
                w = torch.rand((B, Lq, 1), generator=gen, dtype=torch.float64) * 0.3 + 0.05
                refp = torch.cat([c, w], -1)[:, :, None].expand(B, Lq, L, 2)
            refp = refp.contiguous()
            query = torch.randn((B, Lq, qdim), generator=gen, dtype=torch.float64).requires_grad_(True)
            flat = torch.randn((B, S, d_model), generator=gen, dtype=torch.float64).requires_grad_(True)
            m.zero_grad()
            if name == "attn":
                with _zeros_padding(ref):
                    y = m(query, refp, flat, shp, start, mask)
            else:
                y = m(query, refp, flat, shp, start, mask)
            gout = torch.randn(y.shape, generator=gen, dtype=torch.float64)
            y.backward(gout)
            entry[case] = dict(query=query.detach(), reference_points=refp, input_flatten=flat.detach(),
                               grad_out=gout, output=y.detach(), grad_query=query.grad, grad_input_flatten=flat.grad,
                               param_grads={k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
        entry["padding_mask"] = mask
        res[name] = entry
    return res


def transformer_bf16_case(ref):
    """transformer_f64's model and inputs, run by the reference in fp32 under
    ``torch.autocast('cpu', torch.bfloat16)``: the bench's precision regime executed by the
    reference itself (grid_sample stays fp32 there: it is on autocast's promote list)."""
    g = torch.load(os.path.join(HERE, "transformer_f64.pt"), weights_only=True)
    d_model, heads = 64, 4
    pos_embed = ref.embedding_layers.PositionEmbeddingVideoSine(d_model // 2, normalize=True)
    base = ref.base_encoder.BaseEncoder(4, d_model, d_model)
    tr = ref.uni.DeformableTransformer(d_model=d_model, num_head=heads, num_encoder_layers=2, num_decoder_layers=2,
                                       dim_feedforward=128, dropout=0.0, return_intermediate_dec=True,
                                       num_feature_levels=4, dec_n_points=4, enc_n_points=4)
    qe = torch.nn.Embedding(g["state_dicts"]["query_embedding"]["weight"].shape[0], d_model * 2)
    named = {"pos_embed": pos_embed, "base_encoder": base, "transformer": tr, "query_embedding": qe}
    for n, m in named.items():
        m.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in g["state_dicts"][n].items()})
    video = g["video"].float().requires_grad_(True)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        srcs, masks, pos = base(video, g["mask"], g["durations"].float(), pos_embed)
        src_flatten, shapes, starts, valid, lvl_pos, mask_flatten = tr.prepare_encoder_inputs(srcs, masks, pos)
        memory = tr.forward_encoder(src_flatten, shapes, starts, valid, lvl_pos, mask_flatten)
        B = video.shape[0]
        qmask = torch.ones(B, qe.weight.shape[0], dtype=torch.bool)
        _, tgt, refp, qpos = tr.prepare_decoder_input_query(B, qe.weight)
        hs, inter = tr.forward_decoder(tgt, refp, memory, shapes, starts, valid, qpos, mask_flatten, qmask, False)
    loss = (hs.float() * g["w_hs"].float()).sum() + (memory.float() * g["w_mem"].float()).sum()
    loss.backward()
    rel = lambda a, b: ((a.double() - b).norm() / b.norm()).item()  # noqa: E731
    print("reference bf16-autocast vs its fp64 run: memory %.3e hs %.3e grad_video %.3e" % (
        rel(memory.detach(), g["memory"]), rel(hs.detach(), g["hs"]), rel(video.grad, g["grad_video"])))
    return dict(memory=memory.detach().float(), hs=hs.detach().float(), memory_dtype=str(memory.dtype),
                grad_video=video.grad.clone(),
                param_grads={n: {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None}
                             for n, m in named.items()})


D256 = dict(d_model=256, heads=8, ff=1024, Q=20, B=2, T=64, seed=97)


def d256_inputs():
    """Inputs of transformer_bf16_d256 (regenerable: the GPU test calls this too)."""
    c = D256
    gen = torch.Generator().manual_seed(c["seed"])
    video = torch.randn((c["B"], c["T"], c["d_model"]), generator=gen, dtype=torch.float64).float()
    mask = torch.zeros(c["B"], c["T"], dtype=torch.bool)
    mask[1, 48:] = True
    durations = torch.tensor([37.5, 120.25], dtype=torch.float32)
    return video, mask, durations, gen


def transformer_bf16_d256_case(ref):
    """The bench's composition at a shape where its fused paths engage (d % 256 == 0, >= 2 decoder
    layers): PositionEmbeddingVideoSine + BaseEncoder + DeformableTransformer (2 + 2 layers, 8 heads,
    ff 1024, dropout 0) on T=64, B=2 with one padded clip, run by the reference in fp64 (the truth)
    and in fp32 under torch.autocast('cpu', bfloat16) (the reference's own bf16 run: grid_sample
    stays fp32 there, autocast promotes it).  Parameters from regen_parameters; loss
    (hs * w_hs).sum() + (memory * w_mem).sum()."""
    c = D256
    d, heads, Q = c["d_model"], c["heads"], c["Q"]
    named = torch.nn.ModuleDict(dict(
        pos_embed=ref.embedding_layers.PositionEmbeddingVideoSine(d // 2, normalize=True),
        base_encoder=ref.base_encoder.BaseEncoder(4, d, d),
        transformer=ref.uni.DeformableTransformer(d_model=d, num_head=heads, num_encoder_layers=2,
                                                  num_decoder_layers=2, dim_feedforward=c["ff"], dropout=0.0,
                                                  return_intermediate_dec=True, num_feature_levels=4,
                                                  dec_n_points=4, enc_n_points=4),
        query_embedding=torch.nn.Embedding(Q, 2 * d)))
    sums = regen_parameters(named, c["seed"])
    video, mask, durations, gen = d256_inputs()
    w_hs = torch.randn((2, c["B"], Q, d), generator=gen, dtype=torch.float64).float()
    w_mem = torch.randn((c["B"], 120, d), generator=gen, dtype=torch.float64).float()

    def run(mods, dtype, autocast):
        v = video.to(dtype).requires_grad_(True)
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
            srcs, masks, pos = mods["base_encoder"](v, mask, durations.to(dtype), mods["pos_embed"])
            tr = mods["transformer"]
            src_flatten, shapes, starts, valid, lvl_pos, mask_flatten = tr.prepare_encoder_inputs(srcs, masks, pos)
            memory = tr.forward_encoder(src_flatten, shapes, starts, valid, lvl_pos, mask_flatten)
            qmask = torch.ones(c["B"], Q, dtype=torch.bool)
            _, tgt, refp, qpos = tr.prepare_decoder_input_query(c["B"], mods["query_embedding"].weight)
            hs, _ = tr.forward_decoder(tgt, refp, memory, shapes, starts, valid, qpos, mask_flatten, qmask, False)
        loss = (hs.to(dtype) * w_hs.to(dtype)).sum() + (memory.to(dtype) * w_mem.to(dtype)).sum()
        loss.backward()
        return dict(memory=memory.detach().float(), hs=hs.detach().float(), grad_video=v.grad.float(),
                    grads=sampled_grads(dict(mods.items())))

    import copy
    m64 = copy.deepcopy(named).double()
    torch.set_default_dtype(torch.float64)  # the duration embedding allocates with the default dtype
    try:
        truth = run(m64, torch.float64, False)
    finally:
        torch.set_default_dtype(torch.float32)
    bf16 = run(named, torch.float32, True)
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    print("d256: reference bf16 vs fp64: memory %.3e hs %.3e grad_video %.3e" % (
        rel(bf16["memory"], truth["memory"]), rel(bf16["hs"], truth["hs"]),
        rel(bf16["grad_video"], truth["grad_video"])))
    return dict(config={k: torch.tensor(v) for k, v in c.items()}, param_abs_sums=sums, w_hs=w_hs, w_mem=w_mem,
                truth=truth, bf16=bf16)


SPARSE256 = dict(d_model=256, heads=4, ff=1024, Q=10, B=2, T=64, rho_pct=30, seed0=300)


def sparse256_inputs(seed):
    """Inputs of sparse_bf16_d256 (regenerable: the GPU test calls this too): two clips of T=64
    features, the second padded from frame 40."""
    c = SPARSE256
    gen = torch.Generator().manual_seed(seed)
    video = torch.randn((c["B"], c["T"], c["d_model"]), generator=gen, dtype=torch.float64).float()
    mask = torch.zeros(c["B"], c["T"], dtype=torch.bool)
    mask[1, 40:] = True
    durations = torch.tensor([41.0, 97.5], dtype=torch.float32)
    return video, mask, durations, gen


def sparse256_modules(ref_or_ours, sparse_cls, embedding_layers, base_encoder):
    c = SPARSE256
    d = c["d_model"]
    return torch.nn.ModuleDict(dict(
        pos_embed=embedding_layers.PositionEmbeddingVideoSine(d // 2, normalize=True),
        base_encoder=base_encoder.BaseEncoder(4, d, d),
        transformer=sparse_cls(d_model=d, num_head=c["heads"], num_encoder_layers=2, num_decoder_layers=2,
                               dim_feedforward=c["ff"], dropout=0.0, return_intermediate_dec=True,
                               num_feature_levels=4, dec_n_points=4, enc_n_points=4, rho=c["rho_pct"] / 100),
        query_embedding=torch.nn.Embedding(c["Q"], 2 * d)))


def sparse256_forward(mods, video, mask, durations):
    """The Sparse-DETR transformer's training forward (reference
    models/sparse/unimodal_sparse_deformable_transformer.py:152-290): BaseEncoder pyramid, mask
    predictor + top-k token selection (rho), sparse encoder over the selected tokens scattered back
    into the memory, query decoder.  Returns (memory, hs, mask_prediction, topk, sparse_token_nums)."""
    c = SPARSE256
    srcs, masks, pos = mods["base_encoder"](video, mask, durations, mods["pos_embed"])
    tr = mods["transformer"]
    (src_flatten, shapes, starts, valid, lvl_pos, mask_flatten, proposals, topk, mask_pred,
     stn) = tr.prepare_encoder_inputs(srcs, masks, pos)
    memory = tr.forward_encoder(src_flatten, shapes, starts, valid, lvl_pos, mask_flatten, proposals, topk, stn)[0]
    B = video.shape[0]
    qmask = torch.ones(B, c["Q"], dtype=torch.bool, device=video.device)
    _, tgt, refp, qpos = tr.prepare_decoder_input_query(B, mods["query_embedding"].weight)
    hs = tr.forward_decoder(tgt, refp, memory, shapes, starts, valid, qpos, mask_flatten, qmask, False)[0]
    return memory, hs, mask_pred, topk, stn


def topk_sets(topk, stn):
    """Each clip's selected tokens as a sorted tensor (the encoder refines topk[i, :stn[i]])."""
    return [topk[i, :int(stn[i])].sort().values for i in range(topk.shape[0])]


def topk_margin(mask_pred, stn):
    """Smallest gap, over clips, between the last selected and the first unselected fp64 score, in
    units of the bf16 spacing at that magnitude (a margin of many units: bf16 rounding cannot swap
    the two)."""
    m = float("inf")
    for i in range(mask_pred.shape[0]):
        s = mask_pred[i].double().sort(descending=True).values
        k = int(stn[i])
        if k >= s.numel():
            continue
        gap = (s[k - 1] - s[k]).item()
        mag = max(abs(s[k - 1].item()), abs(s[k].item()), 1e-30)
        ulp = 2.0 ** (math.floor(math.log2(mag)) - 7)
        m = min(m, gap / ulp)
    return m


def sparse_bf16_d256_case(ref):
    """The reference's default-active Sparse-DETR transformer (rho 0.3, 2 + 2 layers, d=256, 4 heads of
    64 channels: the bench kernels' D) behind PositionEmbeddingVideoSine + BaseEncoder, T=64, B=2 with
    one padded clip, dropout 0, in fp64 (the truth) and in fp32 under torch.autocast('cpu', bfloat16)
    (the reference's own bf16 run).  Loss (hs w_hs).sum() + (memory w_mem).sum() + (mask_pred w_mp).sum().
    The seed is the first from seed0 whose bf16 run selects the fp64 run's tokens in every clip with a
    score margin of at least 16 bf16 spacings (so a bf16 implementation can be held to that selection)."""
    c = SPARSE256
    Q, d = c["Q"], c["d_model"]

    def run(mods, video, mask, durations, w, dtype, autocast):
        v = video.to(dtype).requires_grad_(True)
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
            memory, hs, mask_pred, topk, stn = sparse256_forward(mods, v, mask, durations.to(dtype))
        loss = ((hs.to(dtype) * w[0].to(dtype)).sum() + (memory.to(dtype) * w[1].to(dtype)).sum()
                + (mask_pred.to(dtype) * w[2].to(dtype)).sum())
        loss.backward()
        return dict(memory=memory.detach().float(), hs=hs.detach().float(), mask_pred=mask_pred.detach().float(),
                    topk=topk, stn=stn, grad_video=v.grad.float(), loss=loss.detach().double(),
                    grads=sampled_grads(dict(mods.items())))

    import copy
    for seed in range(c["seed0"], c["seed0"] + 50):
        named = sparse256_modules(ref, ref.sparse.SparseDeformableTransformer, ref.embedding_layers, ref.base_encoder)
        sums = regen_parameters(named, seed)
        video, mask, durations, gen = sparse256_inputs(seed)
        w = [torch.randn(sh, generator=gen, dtype=torch.float64).float()
             for sh in ((2, c["B"], Q, d), (c["B"], 120, d), (c["B"], 120))]
        m64 = copy.deepcopy(named).double()
        torch.set_default_dtype(torch.float64)
        try:
            truth = run(m64, video, mask, durations, w, torch.float64, False)
        finally:
            torch.set_default_dtype(torch.float32)
        bf16 = run(named, video, mask, durations, w, torch.float32, True)
        same = all(torch.equal(a, b) for a, b in zip(topk_sets(truth["topk"], truth["stn"]),
                                                      topk_sets(bf16["topk"], bf16["stn"])))
        margin = topk_margin(truth["mask_pred"], truth["stn"])
        print(f"sparse256 seed {seed}: bf16 selects the fp64 tokens {same}, margin {margin:.1f} bf16 spacings")
        if same and margin >= 16:
            break
    else:
        raise RuntimeError("no seed with a clear top-k margin")
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    print("sparse256: reference bf16 vs fp64: memory %.3e hs %.3e mask_pred %.3e grad_video %.3e" % (
        rel(bf16["memory"], truth["memory"]), rel(bf16["hs"], truth["hs"]), rel(bf16["mask_pred"], truth["mask_pred"]),
        rel(bf16["grad_video"], truth["grad_video"])))
    cfg = dict(c, seed=seed)
    return dict(config={k: torch.tensor(v) for k, v in cfg.items()}, param_abs_sums=sums, weights=w,
                margin=torch.tensor(margin), truth=truth, bf16=bf16)


MM256 = dict(d_model=256, heads=4, ff=1024, Q=10, B=2, T=64, Ta=16, seed=131)


def mm256_inputs():
    """Inputs of multimodal_bf16_d256 (regenerable: the GPU test calls this too): video (B, 64, d) and
    audio (B, 16, d) features, the second clip padded from video frame 48 / audio frame 12."""
    c = MM256
    gen = torch.Generator().manual_seed(c["seed"])
    video = torch.randn((c["B"], c["T"], c["d_model"]), generator=gen, dtype=torch.float64).float()
    audio = torch.randn((c["B"], c["Ta"], c["d_model"]), generator=gen, dtype=torch.float64).float()
    vmask = torch.zeros(c["B"], c["T"], dtype=torch.bool)
    vmask[1, 48:] = True
    amask = torch.zeros(c["B"], c["Ta"], dtype=torch.bool)
    amask[1, 12:] = True
    durations = torch.tensor([52.5, 133.75], dtype=torch.float32)
    return video, vmask, audio, amask, durations, gen


def mm256_modules(mm_cls, embedding_layers, base_encoder):
    """The multimodal stack of MultimodalDeformableDVC's proposal path (multimodal_deformable_dvc.py:
    112-170): one PositionEmbeddingVideoSine and one BaseEncoder shared by the video and audio
    streams, MultimodalDeformableTransformer (2 + 2 layers, d=256, 4 heads of 64, ff 1024, dropout 0)."""
    c = MM256
    d = c["d_model"]
    return torch.nn.ModuleDict(dict(
        pos_embed=embedding_layers.PositionEmbeddingVideoSine(d // 2, normalize=True),
        base_encoder=base_encoder.BaseEncoder(4, d, d),
        transformer=mm_cls(d_model=d, num_head=c["heads"], num_encoder_layers=2, num_decoder_layers=2,
                           dim_feedforward=c["ff"], dropout=0.0, return_intermediate_dec=True, num_feature_levels=4,
                           dec_n_points=4, enc_n_points=4),
        query_embedding=torch.nn.Embedding(c["Q"], 2 * d)))


def mm256_forward(mods, video, vmask, audio, amask, durations):
    """Reference multimodal_deformable_transformer.py:237-277 (encoder: per layer video->video,
    audio->audio and both cross-modal MSDA calls through the shared layers) and :380-432 (decoder:
    cross-attention into both memories + the fusion bridge), behind the shared BaseEncoder.
    Returns (memory_video, memory_audio, hs)."""
    tr = mods["transformer"]
    v_srcs, v_masks, v_pos = mods["base_encoder"](video, vmask, durations, mods["pos_embed"])
    a_srcs, a_masks, a_pos = mods["base_encoder"](audio, amask, durations, mods["pos_embed"])
    v = tr.prepare_encoder_inputs(v_srcs, v_masks, v_pos)
    a = tr.prepare_encoder_inputs(a_srcs, a_masks, a_pos)
    mem_v, mem_a = tr.forward_encoder(*v, *a)
    B = video.shape[0]
    qw = mods["query_embedding"].weight
    qmask = torch.ones(B, qw.shape[0], dtype=torch.bool, device=video.device)
    _, tgt, refp, qpos = tr.prepare_decoder_input_query(B, qw)
    hs, _ = tr.forward_decoder(tgt, refp, qpos, qmask, mem_v, v[1], v[2], v[3], v[5], mem_a, a[1], a[2], a[3], a[5],
                               False)
    return mem_v, mem_a, hs


def multimodal_bf16_d256_case(ref):
    """configs[2]'s composition at a size where the bench's fused bf16 paths engage (d % 256 == 0,
    2 + 2 layers): the shared BaseEncoder over video (T=64) and audio (T=16) and the reference's
    MultimodalDeformableTransformer (4 heads of 64 channels: the bench kernels' D), B=2 with one padded
    clip, dropout 0 — in fp64 (the truth) and in fp32 under torch.autocast('cpu', bfloat16) (the
    reference's own bf16 run).  Loss (hs w_hs).sum() + (memory_video w_v).sum() + (memory_audio w_a).sum().
    Parameters from regen_parameters; gradients on fixed samples plus their norms."""
    import copy
    c = MM256
    named = mm256_modules(ref.mm.MultimodalDeformableTransformer, ref.embedding_layers, ref.base_encoder)
    sums = regen_parameters(named, c["seed"])
    video, vmask, audio, amask, durations, gen = mm256_inputs()
    Sv = sum(c["T"] >> l for l in range(4))
    Sa = sum(c["Ta"] >> l for l in range(4))
    w = [torch.randn(sh, generator=gen, dtype=torch.float64).float()
         for sh in ((2, c["B"], c["Q"], c["d_model"]), (c["B"], Sv, c["d_model"]), (c["B"], Sa, c["d_model"]))]

    def run(mods, dtype, autocast):
        v = video.to(dtype).requires_grad_(True)
        a = audio.to(dtype).requires_grad_(True)
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
            mem_v, mem_a, hs = mm256_forward(mods, v, vmask, a, amask, durations.to(dtype))
        loss = ((hs.to(dtype) * w[0].to(dtype)).sum() + (mem_v.to(dtype) * w[1].to(dtype)).sum()
                + (mem_a.to(dtype) * w[2].to(dtype)).sum())
        loss.backward()
        return dict(memory_video=mem_v.detach().float(), memory_audio=mem_a.detach().float(), hs=hs.detach().float(),
                    grad_video=v.grad.float(), grad_audio=a.grad.float(), loss=loss.detach().double(),
                    grads=sampled_grads(dict(mods.items())))

    m64 = copy.deepcopy(named).double()
    torch.set_default_dtype(torch.float64)  # the duration embedding allocates with the default dtype
    try:
        truth = run(m64, torch.float64, False)
    finally:
        torch.set_default_dtype(torch.float32)
    bf16 = run(named, torch.float32, True)
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    print("mm256: reference bf16 vs fp64: " + " ".join(
        f"{k} {rel(bf16[k], truth[k]):.3e}" for k in ("memory_video", "memory_audio", "hs", "grad_video", "grad_audio")))
    return dict(config={k: torch.tensor(v) for k, v in c.items()}, param_abs_sums=sums, weights=w, truth=truth,
                bf16=bf16)


CAPTION = dict(vocab=10000, seq_len=20, d_model=512, depth=2, heads=8, N=6, K=40, seed=101, head_scale=8.0,
               bos=2, eos=3, pad=1)


def caption_inputs():
    """Captions, memories and masks of caption_bf16 (regenerable: the GPU test calls this too)."""
    c = CAPTION
    gen = torch.Generator().manual_seed(c["seed"])
    L = c["seq_len"] - 1
    tgt = torch.randint(4, c["vocab"], (c["N"], L), generator=gen)
    tgt[:, 0] = c["bos"]
    for n, end in enumerate([19, 12, 7, 19, 15, 10]):
        if end < L:
            tgt[n, end] = c["eos"]
            tgt[n, end + 1:] = c["pad"]
    memory = torch.randn((c["N"], c["K"], c["d_model"]), generator=gen, dtype=torch.float64).float()
    kmask = torch.zeros(c["N"], c["K"], dtype=torch.bool)
    kmask[1, 30:] = True
    kmask[4, 11:] = True
    return tgt, memory, kmask


def caption_masks(captions, pad):
    """make_padding_mask / make_tgt_mask of the reference DVC (unimodal_deformable_dvc.py:384-431)."""
    padding = captions == pad
    L = captions.shape[1]
    look = 1 - torch.tril(torch.ones((L, L), device=captions.device))
    return padding, torch.maximum(padding.unsqueeze(1).unsqueeze(1), look).bool()


def decode_gap(full64, caps, pad, eos, faster_eval):
    """How far a decoded caption path is from greedy under an fp64 model: the largest
    log p(argmax) - log p(chosen) over the words the loop chose, each step evaluated on the
    loop's own input at that step (words >= w still <pad>).  0 for the fp64 greedy path."""
    worst = 0.0
    n, L = caps.shape
    done = torch.zeros(n, dtype=torch.bool, device=caps.device)
    with torch.no_grad():
        for w in range(1, L):
            inp = caps.clone()
            inp[:, w:] = pad
            pmask, tmask = caption_masks(inp, pad)
            lp = torch.log(full64(inp, pmask, tmask)[:, w].double() + 1e-300)
            chosen = caps[:, w].long()
            g = lp.max(-1).values - lp.gather(-1, chosen[:, None])[:, 0]
            live = torch.ones(n, dtype=torch.bool, device=caps.device) if faster_eval else ~done
            if live.any():
                worst = max(worst, g[live].max().item())
            if not faster_eval:
                done = done | (live & (chosen == eos))
    return worst


def caption_bf16_case(ref):
    """The reference's UnimodalCaptionDecoder (models/unimodal_caption_decoder.py:19-107) at config
    scale (d=512, 8 heads, vocab 10000, seq_len 20; depth 2, post-norm, dropout 0), parameters from
    regen_parameters (head weights x8: confident argmax, so greedy decodes have no near-ties):
    teacher-forced forward with the DVC's masks and the gradients of -sum p(target); the reference's
    greedy re-decode loop (unimodal_deformable_dvc.py:304-354, exact and faster_eval) — each in
    fp64 and under torch.autocast('cpu', bfloat16).  The caption decoder is called with the
    argument order its signature declares (tgt_mask, memory_mask, tgt_padding_mask)."""
    import models.unimodal_caption_decoder as ref_ucd  # noqa: E402
    c = CAPTION
    torch.manual_seed(c["seed"])
    dec = ref_ucd.UnimodalCaptionDecoder(c["vocab"], seq_len=c["seq_len"], d_model=c["d_model"], depth=c["depth"],
                                         num_heads=c["heads"], mlp_ratio=4, qkv_bias=True, pre_norm=False,
                                         return_intermediate=True)
    sums = regen_parameters(dec, c["seed"], scale={"head.weight": c["head_scale"]})
    tgt, memory, kmask = caption_inputs()
    padding, tgt_mask = caption_masks(tgt, c["pad"])
    gen = torch.Generator().manual_seed(c["seed"] + 1)
    vsub = torch.randperm(c["vocab"], generator=gen)[:256].sort().values
    nxt = torch.cat([tgt[:, 1:], torch.full((c["N"], 1), c["eos"])], 1)  # the word each position predicts
    live = nxt != c["pad"]

    def forward(m, dtype, autocast):
        mem = memory.to(dtype).requires_grad_(True)
        m.zero_grad()
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
            out = m(tgt, mem, tgt_mask=tgt_mask, memory_mask=kmask[:, None, None, :], tgt_padding_mask=padding)
        out = out.to(dtype)
        p_t = out.gather(-1, nxt[None, :, :, None].expand(out.shape[0], -1, -1, 1))[..., 0]
        loss = -(p_t * live).sum()  # smooth in p (a log would weigh tiny, rounding-dominated p_t)
        loss.backward()
        return dict(argmax=out.argmax(-1), p_target=p_t.detach().float(), probs_sub=out[..., vsub].detach().float(),
                    grad_memory=mem.grad.float(), grads=sampled_grads({"decoder": m}))

    def decode(m, dtype, autocast, faster_eval):
        mem = memory.to(dtype)
        caps = torch.ones([c["N"], c["seq_len"] - 1], dtype=torch.int32)
        caps[:, 0] = c["bos"]
        done = []
        with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
            for w in range(1, c["seq_len"] - 1):
                pmask, tmask = caption_masks(caps, c["pad"])
                out = m(caps, mem, tgt_mask=tmask, memory_mask=kmask[:, None, None, :], tgt_padding_mask=pmask)
                top = torch.argmax(out[-1], dim=2)
                if faster_eval:
                    caps[:, w] = top[:, w]
                else:
                    for i in range(c["N"]):
                        if i not in done:
                            caps[i, w] = top[i, w]
                            if top[i, w] == c["eos"]:
                                done.append(i)
        return caps

    import copy
    d64 = copy.deepcopy(dec).double()
    res = dict(config={k: torch.tensor(v) for k, v in c.items()}, param_abs_sums=sums, vocab_sample=vsub,
               truth=forward(d64, torch.float64, False), bf16=forward(dec, torch.float32, True))
    for fe in (False, True):
        key = "faster" if fe else "exact"
        truth, b16 = decode(d64, torch.float64, False, fe), decode(dec, torch.float32, True, fe)
        gap = decode_gap(lambda cp, pm, tm: d64(cp, memory.double(), tgt_mask=tm,
                                                memory_mask=kmask[:, None, None, :], tgt_padding_mask=pm)[-1],
                         b16, c["pad"], c["eos"], fe)
        res["decode_" + key] = dict(truth=truth, bf16=b16, bf16_gap=torch.tensor(gap, dtype=torch.float64))
        print("caption decode %s: reference bf16 == fp64: %s; bf16 path's worst fp64 log-prob gap %.4f" % (
            key, bool(torch.equal(truth, b16)), gap))
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    print("caption: reference bf16 vs fp64: p_target %.3e grad_memory %.3e" % (
        rel(res["bf16"]["p_target"], res["truth"]["p_target"]),
        rel(res["bf16"]["grad_memory"], res["truth"]["grad_memory"])))
    return res


SPARSE_DVC_VOCAB = ['<unk>', '<pad>', '<bos>', '<eos>'] + [f"w{i}" for i in range(26)]


def sparse_dvc_args():
    """Namespaces standing in for cfg.dvc / cfg.dvc.sparse_detr / cfg.dvc.caption (config_dvc_train.py)
    at a small size; dropout 0 so forward and gradients are deterministic."""
    ns = types.SimpleNamespace
    d = 64
    sparse = ns(feature_dim=d, d_model=d, hidden_dim=d, num_heads=4, num_feature_levels=4, dec_n_points=4,
                enc_n_points=4, enc_layers=2, dec_layers=2, transformer_dropout_prob=0.0, transformer_ff_dim=128,
                video_rescale_len=64, rho=0.3, use_enc_aux_loss=True, return_intermediate=True, eff_query_init=True,
                eff_specific_head=True)
    caption = ns(d_model=d, depth=2, num_heads=4, mlp_ratio=4, qkv_bias=True, positional_embedding_dropout=0.0,
                 attention_dropout=0.0, projection_dropout=0.0, bridge_dropout=0.0, mlp_dropout_1=0.0, mlp_dropout_2=0.0,
                 pre_norm=False, model_official=None, weight_init=True, weight_load=False, emb_weights_req_grad=True,
                 return_intermediate=True)
    matcher = ns(cost_class=1, cost_segment=5, cost_giou=2, cost_alpha=0.25, cost_gamma=2.0)
    return dict(d_model=d, num_queries=10, num_classes=20, max_eseq_length=10, seq_len=12, sparse=sparse,
                caption=caption, matcher=matcher)


def sparse_dvc_batch(seed, d, T, dtype, vocab_size, seq_len):
    """engine.py-shaped ``obj`` (dataset/anet_video.py:262-384 collate keys) with 2 clips."""
    gen = torch.Generator().manual_seed(seed)
    B = 2
    video = torch.randn((B, T, d), generator=gen, dtype=torch.float64).to(dtype)
    mask = torch.zeros(B, T, dtype=torch.bool)
    mask[1, (3 * T) // 4:] = True
    durations = torch.tensor([37.5, 121.25], dtype=torch.float32)
    nseg = [3, 2]
    targets, caps = [], []
    for b in range(B):
        c = torch.rand((nseg[b],), generator=gen, dtype=torch.float32) * 0.6 + 0.2
        l = torch.rand((nseg[b],), generator=gen, dtype=torch.float32) * 0.3 + 0.05
        targets.append({'segments': torch.stack([c, l], 1).to(dtype), 'labels': torch.zeros(nseg[b], dtype=torch.long),
                        'masks': None, 'vid_id': f"v{b}"})
    total = sum(nseg)
    cap = torch.full((total, seq_len), 1, dtype=torch.long)
    cap_mask = torch.ones((total, seq_len), dtype=torch.bool)
    for i in range(total):
        n = 4 + i % (seq_len - 5)
        body = torch.randint(4, vocab_size, (n,), generator=gen)
        row = torch.cat([torch.tensor([2]), body, torch.tensor([3])])
        cap[i, :len(row)] = row
        cap_mask[i, :len(row)] = False
    length = torch.tensor([[float(T), durations[b].item(), float(nseg[b])] for b in range(B)], dtype=torch.float32)
    return {'video_tensor': video, 'video_mask': mask, 'video_length': length, 'video_target': targets,
            'cap_tensor': cap, 'cap_mask': cap_mask}


def sparse_dvc_case(ref, seed=71):
    """The reference's UnimodalSparseDVC (models/sparse/unimodal_sparse_dvc.py), the one DVC wrapper
    that runs end to end at HEAD: training forward (heads, Hungarian matching, crop, teacher-forced
    caption decoder) + backward of a weighted sum of its outputs, and the eval-mode greedy decode
    (val_mode one_by_one, faster_eval False and True).  fp64."""
    import models.matcher as ref_matcher  # noqa: E402
    import models.sparse.unimodal_sparse_dvc as ref_sdvc  # noqa: E402
    a = sparse_dvc_args()
    vocab = {w: i for i, w in enumerate(SPARSE_DVC_VOCAB)}
    torch.manual_seed(seed)
    matcher = ref_matcher.build_matcher(a["matcher"])
    model = ref_sdvc.UnimodalSparseDVC(['video'], a["num_queries"], a["d_model"], a["num_classes"], True, matcher,
                                       0.5, a["max_eseq_length"], vocab, a["seq_len"], None, a["sparse"],
                                       a["caption"], use_differentiable_mask=False).double()
    # the duration embedding allocates with the default dtype (embedding_layers.py:222)
    torch.set_default_dtype(torch.float64)
    try:
        _jitter_offsets(model, seed)
        with torch.no_grad():  # move the zero-initialised segment heads off zero so matching is generic
            g = torch.Generator().manual_seed(seed + 1)
            for ffn in (model.segment_embedding_decoder, model.segment_embedding_encoder):
                w = ffn.layers[-1].weight
                w.copy_(torch.randn(w.shape, generator=g, dtype=torch.float64) * 0.2)
        obj = sparse_dvc_batch(seed, a["d_model"], 64, torch.float64, len(vocab), a["seq_len"])
        model.train()
        out, caps, indices, indices_aux, _ = model(obj, is_training=True)
        gen = torch.Generator().manual_seed(seed + 2)
        keys = ("pred_segments", "pred_count", "pred_captions", "backbone_mask_prediction")
        w = {k: torch.randn(out[k].shape, generator=gen, dtype=torch.float64) for k in keys}
        loss = sum((out[k] * w[k]).sum() for k in keys)
        loss = loss + sum((o["pred_segments"] * 0.5).sum() + (o["pred_count"] * 0.25).sum() for o in out["aux_outputs"])
        loss = loss + sum((o["pred_segments"] * 0.3).sum() for o in out["aux_outputs_enc"])
        loss.backward()
        train = dict(out={k: out[k].detach() for k in keys}, captions=caps, weights=w, loss=loss.detach(),
                     indices=[torch.stack(list(t)) for t in indices],
                     indices_aux=[[torch.stack(list(t)) for t in lv] for lv in indices_aux],
                     aux_segments=torch.stack([o["pred_segments"].detach() for o in out["aux_outputs"]]),
                     aux_enc_segments=torch.stack([o["pred_segments"].detach() for o in out["aux_outputs_enc"]]),
                     param_grads={k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None})
        model.eval()
        evals = {}
        with torch.no_grad():
            for fe in (False, True):
                o, caps_e, ind, _, _ = model(obj, is_training=False, faster_eval=fe, val_mode="one_by_one")
                evals["faster" if fe else "exact"] = dict(captions=caps_e, pred_captions=o["pred_captions"],
                                                          indices=[torch.stack(list(t)) for t in ind])
        sd = {k: v for k, v in model.state_dict().items() if not k.endswith("positional_encoding.pos_embedding")}
        return dict(state_dict=_compact(sd), obj={k: v for k, v in obj.items()}, vocab=SPARSE_DVC_VOCAB, train=train,
                    eval=evals)
    finally:
        torch.set_default_dtype(torch.float32)


def deformable_dvc_case(ref, seed=73):
    """The reference's UnimodalDeformableDVC (models/deformable/unimodal_deformable_dvc.py) run with
    its one crashing call fixed: the caption decoder is called positionally as
    (captions, memory, tgt_mask, padding_mask, memory_mask) (:277/:328) against the signature
    (tgt, memory, tgt_mask, memory_mask, tgt_padding_mask) (unimodal_caption_decoder.py:68); the
    instance's decoder ``forward`` is wrapped to swap those two arguments.  Everything else is the
    reference code as written.  use_differentiable_mask=True: with False the forward reads an
    unbound ``pred_memory_mask`` (:264).  Training forward + backward, and eval decode."""
    import models.matcher as ref_matcher  # noqa: E402
    import models.deformable.unimodal_deformable_dvc as ref_ddvc  # noqa: E402
    a = sparse_dvc_args()
    s = a["sparse"]
    detr = types.SimpleNamespace(feature_dim=s.feature_dim, d_model=s.d_model, num_heads=s.num_heads,
                                 num_feature_levels=4, dec_n_points=4, enc_n_points=4, enc_layers=2, dec_layers=2,
                                 transformer_dropout_prob=0.0, transformer_ff_dim=128, video_rescale_len=64,
                                 return_intermediate=True, hidden_dropout_prob=0.0, layer_norm_eps=1e-12)
    vocab = {w: i for i, w in enumerate(SPARSE_DVC_VOCAB)}
    torch.manual_seed(seed)
    matcher = ref_matcher.build_matcher(a["matcher"])
    model = ref_ddvc.UnimodalDeformableDVC(['video'], a["num_queries"], a["d_model"], a["num_classes"], True, matcher,
                                           0.5, a["max_eseq_length"], vocab, a["seq_len"], None, detr, a["caption"],
                                           use_differentiable_mask=True).double()
    dec = model.unimodal_caption_decoder
    real_forward = type(dec).forward
    dec.forward = lambda tgt, memory, tgt_mask=None, arg4=None, arg5=None: real_forward(dec, tgt, memory, tgt_mask,
                                                                                        arg5, arg4)
    torch.set_default_dtype(torch.float64)
    try:
        _jitter_offsets(model, seed)
        with torch.no_grad():
            g = torch.Generator().manual_seed(seed + 1)
            w = model.segment_embedding[0].layers[-1].weight
            w.copy_(torch.randn(w.shape, generator=g, dtype=torch.float64) * 0.2)
        obj = sparse_dvc_batch(seed, a["d_model"], 64, torch.float64, len(vocab), a["seq_len"])
        model.train()
        out, caps, indices, indices_aux, mask = model(obj, is_training=True)
        gen = torch.Generator().manual_seed(seed + 2)
        keys = ("pred_logits", "pred_segments", "pred_count", "pred_captions", "pred_memory_mask")
        w = {k: torch.randn(out[k].shape, generator=gen, dtype=torch.float64) for k in keys}
        loss = sum((out[k] * w[k]).sum() for k in keys)
        loss = loss + sum((o["pred_captions"] * 0.5).sum() + (o["pred_segments"] * 0.5).sum() for o in out["aux_outputs"])
        loss.backward()
        train = dict(out={k: out[k].detach() for k in keys}, captions=caps, weights=w, loss=loss.detach(), mask=mask,
                     indices=[torch.stack(list(t)) for t in indices],
                     indices_aux=[[torch.stack(list(t)) for t in lv] for lv in indices_aux],
                     aux_captions=torch.stack([o["pred_captions"].detach() for o in out["aux_outputs"]]),
                     param_grads={k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None})
        model.eval()
        evals = {}
        with torch.no_grad():
            for fe in (False, True):
                o, caps_e, ind, ind_aux, _ = model(obj, is_training=False, faster_eval=fe)
                evals["faster" if fe else "exact"] = dict(
                    captions=caps_e, pred_captions=o["pred_captions"], indices=[torch.stack(list(t)) for t in ind],
                    aux_captions=torch.stack([x["pred_captions"] for x in o["aux_outputs"]]))
        sd = {k: v for k, v in model.state_dict().items() if not k.endswith("positional_encoding.pos_embedding")}
        return dict(state_dict=_compact(sd), obj=obj, vocab=SPARSE_DVC_VOCAB, train=train, eval=evals)
    finally:
        torch.set_default_dtype(torch.float32)


def mm_caption_decoder_case(ref, seed=79):
    """The reference's MultimodalCaptionDecoder (models/multimodal_caption_decoder.py) and its layer
    (models/modules/layers.py:648-823), executed with the undefined names of HEAD bound to the
    objects they evidently mean — nothing in the files is changed:
      * module globals of multimodal_caption_decoder: ``CapMultimodalCaptionDecoderionDecoder`` (:29) ->
        MultimodalCaptionDecoder, ``MultimodalCaptionDecoderrLayer`` (:42) -> a layer class taking the
        decoder's ``dropout_1`` / ``dropout_2`` as the layer's ``mlp_dropout_1`` / ``mlp_dropout_2``;
      * the layer's ``super(UnimodalCaptionDecoderLayer, self)`` (:667) resolves by making the layer
        class also derive from UnimodalCaptionDecoderLayer (its MRO then reaches nn.Module);
      * instance aliases ``activation`` -> ``activation_layer``, ``cross_attention`` ->
        ``audio_cross_attention``, ``audio_projection_dropout_3`` -> ``projection_dropout_3`` (:760,819,823).
    Post-norm (config pre_norm=False); the pre-norm path cannot run (LayerNorm(d) on a 2d concat, :757)."""
    import models.modules.layers as ref_layers  # noqa: E402
    import models.multimodal_caption_decoder as ref_mcd  # noqa: E402

    class Layer(ref_layers.MultimodalCaptionDecoderLayer, ref_layers.UnimodalCaptionDecoderLayer):
        def __init__(self, d_model, num_heads, mlp_ratio, qkv_bias, attention_dropout, projection_dropout,
                     dropout_1, dropout_2, pre_norm):
            ref_layers.MultimodalCaptionDecoderLayer.__init__(
                self, d_model, num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, attention_dropout=attention_dropout,
                projection_dropout=projection_dropout, mlp_dropout_1=dropout_1, mlp_dropout_2=dropout_2,
                pre_norm=pre_norm)
            # plain attributes (not registered submodules): the state_dict keeps the reference's names
            object.__setattr__(self, "activation", self.activation_layer)
            object.__setattr__(self, "cross_attention", self.audio_cross_attention)
            object.__setattr__(self, "audio_projection_dropout_3", self.projection_dropout_3)

        forward = ref_layers.MultimodalCaptionDecoderLayer.forward

    ref_mcd.CapMultimodalCaptionDecoderionDecoder = ref_mcd.MultimodalCaptionDecoder
    ref_mcd.MultimodalCaptionDecoderrLayer = Layer
    torch.manual_seed(seed)
    V, d, N, L, Kv, Ka = 30, 64, 3, 8, 20, 12
    dec = ref_mcd.MultimodalCaptionDecoder(V, seq_len=L, d_model=d, depth=2, num_heads=4, mlp_ratio=4, qkv_bias=True,
                                           pre_norm=False, return_intermediate=True).double()
    gen = torch.Generator().manual_seed(seed)
    with torch.no_grad():  # LayerNorm affine parameters off their (1, 0) init
        for name, p in dec.named_parameters():
            if "layer_norm" in name:
                p.add_(torch.randn(p.shape, generator=gen, dtype=torch.float64) * 0.1)
    tgt = torch.randint(4, V, (N, L), generator=gen)
    tgt[:, 0] = 2
    tgt[0, 6:] = 1
    tgt[2, 4:] = 1
    pad = tgt == 1
    vm = torch.randn((N, Kv, d), generator=gen, dtype=torch.float64).requires_grad_(True)
    am = torch.randn((N, Ka, d), generator=gen, dtype=torch.float64).requires_grad_(True)
    vmask = torch.zeros(N, Kv, dtype=torch.bool)
    vmask[1, 11:] = True
    amask = torch.zeros(N, Ka, dtype=torch.bool)
    amask[0, 5:] = True
    look = torch.ones(L, L, dtype=torch.bool).triu(1)
    out = dec(tgt=tgt, video_memory=vm, audio_memory=am, tgt_mask=look, video_memory_mask=None, audio_memory_mask=None,
              tgt_padding_mask=pad, video_memory_padding_mask=vmask, audio_memory_padding_mask=amask)
    w = torch.randn(out.shape, generator=gen, dtype=torch.float64)
    (out * w).sum().backward()
    sd = {k: v for k, v in dec.state_dict().items() if not k.endswith("positional_encoding.pos_embedding")}
    return dict(state_dict=_compact(sd), tgt=tgt, video_memory=vm.detach(), audio_memory=am.detach(),
                video_mask=vmask, audio_mask=amask, out=out.detach(), w=w, grad_video=vm.grad, grad_audio=am.grad,
                param_grads={k: p.grad.clone() for k, p in dec.named_parameters() if p.grad is not None})


def mm_dvc_args():
    a = sparse_dvc_args()
    s = a["sparse"]
    detr = types.SimpleNamespace(feature_dim=s.feature_dim, d_model=s.d_model, num_heads=s.num_heads,
                                 num_feature_levels=4, dec_n_points=4, enc_n_points=4, enc_layers=2, dec_layers=2,
                                 transformer_dropout_prob=0.0, transformer_ff_dim=128, video_rescale_len=64,
                                 audio_rescale_len=16, return_intermediate=True, rho=0.0, use_enc_aux_loss=False)
    cap = types.SimpleNamespace(**vars(a["caption"]), dropout_1=0.0, dropout_2=0.0)
    return a, detr, cap


def mm_dvc_case(ref, seed=83):
    """The reference's MultimodalDeformableDVC (models/deformable/multimodal_deformable_dvc.py) training
    forward + backward, run with the names HEAD leaves undefined bound — nothing in the files changed:
      * module global ``detr_args`` (used in __init__ :63,74,76,88) -> the model arguments;
      * class attribute ``video_num_tokens`` (:95) -> num_tokens; module global ``memory`` (read only
        for ``memory.shape[0]``, the matched-segment count, :284) -> a tensor of that length;
      * the MultimodalCaptionDecoder bindings of mm_caption_decoder_case, and its positional call
        (:320) mapped onto the keyword convention of models/sparse/multimodal_sparse_dvc.py:299-305
        (look-ahead + caption key padding; memory masks as key padding), the only form
        ``nn.MultiheadAttention`` accepts.
    use_differentiable_mask=True: with False the forward reads an unbound mask (:303)."""
    import models.matcher as ref_matcher  # noqa: E402
    import models.deformable.multimodal_deformable_dvc as ref_mdvc  # noqa: E402
    mm_caption_decoder_case(ref, seed)  # installs the caption-decoder bindings
    a, detr, cap = mm_dvc_args()
    vocab = {w: i for i, w in enumerate(SPARSE_DVC_VOCAB)}
    obj = sparse_dvc_batch(seed, a["d_model"], 64, torch.float64, len(vocab), a["seq_len"])
    gen = torch.Generator().manual_seed(seed + 5)
    obj["audio_tensor"] = torch.randn((2, 16, a["d_model"]), generator=gen, dtype=torch.float64)
    obj["audio_mask"] = torch.zeros(2, 16, dtype=torch.bool)
    obj["audio_mask"][1, 13:] = True
    n_segments = sum(len(t["segments"]) for t in obj["video_target"])
    ref_mdvc.detr_args = detr
    ref_mdvc.memory = torch.zeros(n_segments)
    ref_mdvc.MultimodalDeformableDVC.video_num_tokens = 120
    torch.manual_seed(seed)
    matcher = ref_matcher.build_matcher(a["matcher"])
    model = ref_mdvc.MultimodalDeformableDVC(['video', 'audio'], a["num_queries"], a["d_model"], a["num_classes"], True,
                                             matcher, 0.5, a["max_eseq_length"], vocab, a["seq_len"], None, detr, cap,
                                             use_differentiable_mask=True).double()
    dec = model.multimodal_caption_decoder
    real_forward = type(dec).forward
    look = torch.ones(a["seq_len"] - 1, a["seq_len"] - 1, dtype=torch.bool).triu(1)

    def positional_call(captions, video_memory, audio_memory, tgt_mask, padding_mask, vmask, amask):
        return real_forward(dec, captions, video_memory, audio_memory, tgt_mask=look, tgt_padding_mask=padding_mask,
                            video_memory_padding_mask=vmask[:, 0, 0, :], audio_memory_padding_mask=amask[:, 0, 0, :])

    dec.forward = positional_call
    torch.set_default_dtype(torch.float64)
    try:
        _jitter_offsets(model, seed)
        with torch.no_grad():
            g = torch.Generator().manual_seed(seed + 1)
            w = model.segment_embedding[0].layers[-1].weight
            w.copy_(torch.randn(w.shape, generator=g, dtype=torch.float64) * 0.2)
        model.train()
        out, caps, indices, indices_aux, vmask, amask = model(obj, is_training=True)
        gen = torch.Generator().manual_seed(seed + 2)
        keys = ("pred_logits", "pred_segments", "pred_count", "pred_captions", "video_pred_memory_mask",
                "audio_pred_memory_mask")
        w = {k: torch.randn(out[k].shape, generator=gen, dtype=torch.float64) for k in keys}
        loss = sum((out[k] * w[k]).sum() for k in keys)
        loss = loss + sum((o["pred_captions"] * 0.5).sum() + (o["pred_segments"] * 0.5).sum() for o in out["aux_outputs"])
        loss.backward()
        sd = {k: v for k, v in model.state_dict().items() if not k.endswith("positional_encoding.pos_embedding")}
        return dict(state_dict=_compact(sd), obj=obj, vocab=SPARSE_DVC_VOCAB, out={k: out[k].detach() for k in keys},
                    captions=caps, weights=w, loss=loss.detach(), video_mask=vmask, audio_mask=amask,
                    indices=[torch.stack(list(t)) for t in indices],
                    indices_aux=[[torch.stack(list(t)) for t in lv] for lv in indices_aux],
                    aux_captions=torch.stack([o["pred_captions"].detach() for o in out["aux_outputs"]]),
                    param_grads={k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None})
    finally:
        torch.set_default_dtype(torch.float32)


DVC256 = dict(d_model=256, heads=4, ff=1024, enc_layers=2, dec_layers=2, caption_depth=2, num_queries=10,
              num_classes=20, T=64, seq_len=12, seed=89)


def dvc256_args():
    """Namespaces of cfg.dvc / cfg.dvc.detr / cfg.dvc.caption (config_dvc_train.py) at d=256, 8 heads,
    2 + 2 layers, ff 1024, T=64, caption depth 2; dropout 0 (shared by the fixture and its GPU test)."""
    c = DVC256
    ns = types.SimpleNamespace
    d = c["d_model"]
    detr = ns(feature_dim=d, d_model=d, num_heads=c["heads"], num_feature_levels=4, dec_n_points=4, enc_n_points=4,
              enc_layers=c["enc_layers"], dec_layers=c["dec_layers"], transformer_dropout_prob=0.0,
              transformer_ff_dim=c["ff"], video_rescale_len=c["T"], return_intermediate=True, hidden_dropout_prob=0.0,
              layer_norm_eps=1e-12)
    caption = ns(d_model=d, depth=c["caption_depth"], num_heads=c["heads"], mlp_ratio=4, qkv_bias=True,
                 positional_embedding_dropout=0.0, attention_dropout=0.0, projection_dropout=0.0, bridge_dropout=0.0,
                 mlp_dropout_1=0.0, mlp_dropout_2=0.0, pre_norm=False, model_official=None, weight_init=True,
                 weight_load=False, emb_weights_req_grad=True, return_intermediate=True)
    matcher = ns(cost_class=1, cost_segment=5, cost_giou=2, cost_alpha=0.25, cost_gamma=2.0)
    return detr, caption, matcher


DVC256_MIN_MARGIN = 0.1

# the last segment-head layer scaled up: spread-out proposals, so every matching is far from a tie
DVC256_SCALE = {"segment_embedding.0.layers.2.weight": 6.0}

DVC256_KEYS = ("pred_logits", "pred_segments", "pred_count", "pred_captions", "pred_memory_mask")


def dvc256_loss(out, w):
    """The fixture's loss: fixed random weights on every training output, plus the aux levels'
    captions and segments (as deformable_dvc_f64), in the weights' dtype."""
    dt = w["pred_logits"].dtype
    loss = sum((out[k].to(dt) * w[k]).sum() for k in DVC256_KEYS)
    return loss + sum((o["pred_captions"].to(dt) * 0.5).sum() + (o["pred_segments"].to(dt) * 0.5).sum()
                      for o in out["aux_outputs"])


def deformable_dvc_bf16_d256_case(ref):
    """The reference's UnimodalDeformableDVC training forward + backward at d=256 (4 heads of 64, 2 + 2 layers,
    ff 1024, caption depth 2, T=64, B=2, 10 queries, dropout 0) — the size at which the bench's fused
    bf16 paths engage — run by the reference in fp64 (the truth) and in fp32 under
    torch.autocast('cpu', bfloat16) (the reference's own bf16 run), with deformable_dvc_f64's one
    argument-order fix of the caption-decoder call.  Parameters from regen_parameters (no state_dict
    stored).  The seed is the first from DVC256['seed'] on at which the bf16 run matches the same
    (clip, prediction) pairs as fp64 on every decoder level with a matching-cost margin of at least
    DVC256_MIN_MARGIN (so our bf16 forward must give that matching too); the GPU test runs the step on those
    pairs (the matching's own arithmetic is pinned in fp64 by deformable_dvc_f64).  The matching
    costs' smallest margin (cost increase when one matched pair is forbidden) is stored."""
    import copy
    import models.matcher as ref_matcher  # noqa: E402
    import models.deformable.unimodal_deformable_dvc as ref_ddvc  # noqa: E402
    c = dict(DVC256)
    detr, caption, mcfg = dvc256_args()
    vocab = {w: i for i, w in enumerate(SPARSE_DVC_VOCAB)}

    def fix_call(model):
        dec = model.unimodal_caption_decoder
        real_forward = type(dec).forward
        dec.forward = lambda tgt, memory, tgt_mask=None, a4=None, a5=None: real_forward(dec, tgt, memory, tgt_mask, a5,
                                                                                        a4)
        return model

    def build():
        matcher = ref_matcher.build_matcher(mcfg)
        return fix_call(ref_ddvc.UnimodalDeformableDVC(['video'], c["num_queries"], c["d_model"], c["num_classes"],
                                                       True, matcher, 0.5, 10, vocab, c["seq_len"], None, detr, caption,
                                                       use_differentiable_mask=True))

    def run(model, obj, w, dtype, autocast):
        model.train()
        model.zero_grad()
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
            out, caps, indices, indices_aux, mask = model(obj, is_training=True)
        loss = dvc256_loss(out, {k: v.to(dtype) for k, v in w.items()})
        loss.backward()
        return dict(out={k: out[k].detach().float() for k in DVC256_KEYS}, loss=loss.detach().double(),
                    aux_captions=torch.stack([o["pred_captions"].detach().float() for o in out["aux_outputs"]]),
                    indices=[torch.stack(list(t)) for t in indices],
                    indices_aux=[[torch.stack(list(t)) for t in lv] for lv in indices_aux],
                    grads=sampled_grads({"dvc": model}))

    for attempt in range(60):
        seed = DVC256["seed"] + attempt
        torch.manual_seed(seed)
        model = build()
        sums = regen_parameters(model, seed, scale=DVC256_SCALE)
        obj32 = sparse_dvc_batch(seed, c["d_model"], c["T"], torch.float32, len(vocab), c["seq_len"])
        gen = torch.Generator().manual_seed(seed + 2)
        with torch.no_grad():
            probe = model(obj32, is_training=True)[0]
        w = {k: torch.randn(probe[k].shape, generator=gen, dtype=torch.float64) for k in DVC256_KEYS}
        m64 = fix_call(copy.deepcopy(model).double())
        obj64 = sparse_dvc_batch(seed, c["d_model"], c["T"], torch.float64, len(vocab), c["seq_len"])
        torch.set_default_dtype(torch.float64)  # the duration embedding allocates with the default dtype
        try:
            truth = run(m64, obj64, w, torch.float64, False)
            margin = min_assignment_margin(m64, obj64)
        finally:
            torch.set_default_dtype(torch.float32)
        bf16 = run(model, obj32, w, torch.float32, True)
        same = all(torch.equal(a, b) for a, b in zip(truth["indices"], bf16["indices"])) and all(
            torch.equal(a, b) for la, lb in zip(truth["indices_aux"], bf16["indices_aux"]) for a, b in zip(la, lb))
        print(f"dvc256 seed {seed}: bf16 matching == fp64: {same}; smallest cost margin {margin:.4f}")
        # a margin well above the bf16 noise of the costs (~0.01 here): any bf16 implementation of the
        # forward must then give the same matching (the GPU test asserts ours does)
        if same and margin >= DVC256_MIN_MARGIN:
            break
    else:
        raise RuntimeError("no seed with the same matching in bf16 and fp64")
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    print("dvc256: reference bf16 vs fp64: " + " ".join(
        f"{k} {rel(bf16['out'][k], truth['out'][k]):.3e}" for k in DVC256_KEYS) + f" loss {rel(bf16['loss'], truth['loss']):.3e}")
    c["seed"] = seed
    return dict(config={k: torch.tensor(v) for k, v in c.items()}, param_abs_sums=sums, weights=w,
                margin=torch.tensor(margin, dtype=torch.float64), truth=truth, bf16=bf16)


def min_assignment_margin(model, obj):
    """How far the fixture's matchings are from a tie: over every decoder level and clip, the smallest
    increase of the optimal assignment cost when one matched (prediction, target) pair is forbidden
    (scipy's solver on the reference matcher's cost, models/matcher.py:64-92, in fp64)."""
    from scipy.optimize import linear_sum_assignment
    from utils.box_ops import generalized_box_iou, segment_cl_to_xy  # noqa: E402
    with torch.no_grad():
        out = model(obj, is_training=True)[0]
    mt = model.matcher
    worst = float("inf")
    for o in [out] + list(out["aux_outputs"]):
        for b, t in enumerate(obj["video_target"]):
            seg, tseg = o["pred_segments"][b].double(), t["segments"].double()
            cost = (mt.cost_segment * torch.cdist(seg, tseg, p=1)
                    - mt.cost_giou * generalized_box_iou(segment_cl_to_xy(seg), segment_cl_to_xy(tseg))).numpy()
            rows, cols = linear_sum_assignment(cost)
            best = cost[rows, cols].sum()
            for r, cc in zip(rows, cols):
                c2 = cost.copy()
                c2[r, cc] = 1e9
                r2, k2 = linear_sum_assignment(c2)
                worst = min(worst, c2[r2, k2].sum() - best)
    return worst


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref = import_reference()
    small = dict(shapes=[32, 16, 8, 4], B=2, M=4, D=8, Lq=20, P=4)
    cases = {
        "op_border_f64": lambda: op_case(ref, torch.float64, seed=1, **small),
        "op_border_f32": lambda: op_case(ref, torch.float32, seed=2, **small),
        "op_border_f32_enc": lambda: op_enc_case(ref),
        "module_f64": lambda: module_case(ref),
        "transformer_f64": lambda: transformer_case(ref),
        "multimodal_f64": lambda: multimodal_case(ref),
        "dam_f32": lambda: dam_case(ref),
        "sparse_f64": lambda: sparse_case(ref),
        "ops_api_f64": lambda: ops_api_case(ref),
        "ops_module_f64": lambda: ops_module_case(ref),
        "transformer_bf16": lambda: transformer_bf16_case(ref),
        "sparse_dvc_f64": lambda: sparse_dvc_case(ref),
        "deformable_dvc_f64": lambda: deformable_dvc_case(ref),
        "mm_caption_decoder_f64": lambda: mm_caption_decoder_case(ref),
        "mm_dvc_f64": lambda: mm_dvc_case(ref),
        "transformer_bf16_d256": lambda: transformer_bf16_d256_case(ref),
        "caption_bf16": lambda: caption_bf16_case(ref),
        "deformable_dvc_bf16_d256": lambda: deformable_dvc_bf16_d256_case(ref),
        "sparse_bf16_d256": lambda: sparse_bf16_d256_case(ref),
        "multimodal_bf16_d256": lambda: multimodal_bf16_d256_case(ref),
    }
    wanted = sys.argv[1:] or list(cases)
    for name, fn in cases.items():
        if any(name.startswith(w) for w in wanted):
            torch.save(fn(), os.path.join(HERE, name + ".pt"))
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".pt"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
