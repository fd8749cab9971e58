"""DVC wrappers and caption decoders behind the reference signatures, against
runs of the reference itself (tests/golden/make_golden.py):

* UnimodalSparseDVC — the reference's default model, end to end as written: heads, Hungarian
  matching, crop, teacher-forced caption decoder, gradients; greedy decode (exact / faster_eval);
* UnimodalDeformableDVC — the reference with its one crashing call (caption-decoder argument
  order) fixed, differentiable mask on (the reference cannot run with it off);
* MultimodalCaptionDecoder — the reference's code with the undefined names of HEAD bound to what
  they evidently mean (make_golden.py::mm_caption_decoder_case);
* MultimodalDeformableDVC — the reference's training forward with HEAD's undefined names bound
  (make_golden.py::mm_dvc_case); its inference (undefined there) runs and returns the engine.py:71 tuple;
* the KV-cached greedy decode of both caption decoders equals the reference's full re-decode loop.

CPU variants run the MSDA core as the oracle restatement (oracle.cpu_model); ``-m gpu`` variants run
the HIP kernels.  fp64 throughout: outputs / gradients 1e-9 relative, matchings and tokens exact."""
import importlib.util
import os
import types

import pytest
import torch

from conftest import PKG, ROOT
from oracle.cpu_model import oracle_core

M = PKG.models
_spec = importlib.util.spec_from_file_location("_mg", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
MG = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MG)  # only its argument / batch builders are used; it imports no reference code


def _vocab():
    return {w: i for i, w in enumerate(MG.SPARSE_DVC_VOCAB)}


def _load(model, sd):
    missing, unexpected = model.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in sd.items()},
                                                strict=False)
    assert not unexpected, unexpected
    assert all(k.endswith("positional_encoding.pos_embedding") for k in missing), missing
    return model


def _obj_to(obj, dev):
    out = {}
    for k, v in obj.items():
        if isinstance(v, torch.Tensor):
            out[k] = v.to(dev)
        elif k == 'video_target':
            out[k] = [{kk: vv.to(dev) if isinstance(vv, torch.Tensor) else vv for kk, vv in t.items()} for t in v]
        else:
            out[k] = v
    return out


def build_sparse_dvc(dev="cpu"):
    a = MG.sparse_dvc_args()
    return M.sparse.unimodal_sparse_dvc.UnimodalSparseDVC(
        ['video'], a["num_queries"], a["d_model"], a["num_classes"], True, M.matcher.build_matcher(a["matcher"]), 0.5,
        a["max_eseq_length"], _vocab(), a["seq_len"], None, a["sparse"], a["caption"]).double().to(dev)


def build_deformable_dvc(dev="cpu", diff_mask=True):
    a = MG.sparse_dvc_args()
    s = a["sparse"]
    detr = types.SimpleNamespace(feature_dim=s.feature_dim, d_model=s.d_model, num_heads=s.num_heads,
                                 num_feature_levels=4, dec_n_points=4, enc_n_points=4, enc_layers=2, dec_layers=2,
                                 transformer_dropout_prob=0.0, transformer_ff_dim=128, video_rescale_len=64,
                                 return_intermediate=True)
    return M.deformable.unimodal_deformable_dvc.UnimodalDeformableDVC(
        ['video'], a["num_queries"], a["d_model"], a["num_classes"], True, M.matcher.build_matcher(a["matcher"]), 0.5,
        a["max_eseq_length"], _vocab(), a["seq_len"], None, detr, a["caption"],
        use_differentiable_mask=diff_mask).double().to(dev)


def _rel(a, b, rel, name=""):
    a, b = a.detach().cpu().double(), b.double()
    err = (a - b).abs().max().item() if a.numel() else 0.0
    assert err <= rel * max(b.abs().max().item() if b.numel() else 0.0, 1e-30) + 1e-12, (name, err)


def _indices_equal(ours, ref):
    assert len(ours) == len(ref)
    for (i, j), r in zip(ours, ref):
        assert torch.equal(torch.stack([i, j]), r)


def _run(model, obj, dev, **kw):
    torch.set_default_dtype(torch.float64)
    try:
        if dev == "cpu":
            with oracle_core(PKG):
                return model(obj, **kw)
        return model(obj, **kw)
    finally:
        torch.set_default_dtype(torch.float32)


def _tol(dev):
    """fp64 models, but the reference computes the sine position embedding in fp32
    (embedding_layers.py:208): GPU vs CPU fp32 sin/cos differ by an ulp, so on the GPU the
    outputs agree to ~1e-7 of fp32 resolution instead of 1e-9 (cf. test_gpu_module.py)."""
    return 1e-9 if dev == "cpu" else 1e-6


def _check_sparse_dvc(golden, dev):
    g = golden("sparse_dvc_f64")
    model = _load(build_sparse_dvc(dev), g["state_dict"])
    obj = _obj_to(g["obj"], dev)
    model.train()
    out, caps, indices, indices_aux, mask = _run(model, obj, dev, is_training=True)
    t = g["train"]
    assert mask is None
    _indices_equal(indices, t["indices"])
    for ours, ref in zip(indices_aux, t["indices_aux"]):
        _indices_equal(ours, ref)
    for k, v in t["out"].items():
        _rel(out[k], v, _tol(dev), k)
    assert torch.equal(caps.cpu(), t["captions"])
    _rel(torch.stack([o["pred_segments"] for o in out["aux_outputs"]]), t["aux_segments"], _tol(dev))
    _rel(torch.stack([o["pred_segments"] for o in out["aux_outputs_enc"]]), t["aux_enc_segments"], _tol(dev))
    w = {k: v.to(dev) for k, v in t["weights"].items()}
    loss = sum((out[k] * w[k]).sum() for k in w)
    loss = loss + sum((o["pred_segments"] * 0.5).sum() + (o["pred_count"] * 0.25).sum() for o in out["aux_outputs"])
    loss = loss + sum((o["pred_segments"] * 0.3).sum() for o in out["aux_outputs_enc"])
    _run_backward(loss, dev)
    _rel(loss, t["loss"], _tol(dev) / 10)
    for k, p in model.named_parameters():
        if k in t["param_grads"]:
            _rel(p.grad, t["param_grads"][k], 10 * _tol(dev), k)
        else:
            assert p.grad is None or p.grad.abs().max() == 0, k
    model.eval()
    with torch.no_grad():
        for name, fe in (("exact", False), ("faster", True)):
            o, caps_e, ind, _, _ = _run(model, obj, dev, is_training=False, faster_eval=fe, val_mode="one_by_one")
            e = g["eval"][name]
            assert torch.equal(caps_e.cpu(), e["captions"]), name
            _rel(o["pred_captions"], e["pred_captions"], _tol(dev), name)
            _indices_equal(ind, e["indices"])


def _run_backward(loss, dev):
    if dev == "cpu":
        with oracle_core(PKG):
            loss.backward()
    else:
        loss.backward()


def _check_deformable_dvc(golden, dev):
    g = golden("deformable_dvc_f64")
    model = _load(build_deformable_dvc(dev), g["state_dict"])
    obj = _obj_to(g["obj"], dev)
    model.train()
    out, caps, indices, indices_aux, mask = _run(model, obj, dev, is_training=True)
    t = g["train"]
    _indices_equal(indices, t["indices"])
    for ours, ref in zip(indices_aux, t["indices_aux"]):
        _indices_equal(ours, ref)
    for k, v in t["out"].items():
        _rel(out[k], v, _tol(dev), k)
    assert torch.equal(caps.cpu(), t["captions"])
    assert torch.equal(mask.cpu(), t["mask"])
    _rel(torch.stack([o["pred_captions"] for o in out["aux_outputs"]]), t["aux_captions"], _tol(dev))
    w = {k: v.to(dev) for k, v in t["weights"].items()}
    loss = sum((out[k] * w[k]).sum() for k in w)
    loss = loss + sum((o["pred_captions"] * 0.5).sum() + (o["pred_segments"] * 0.5).sum() for o in out["aux_outputs"])
    _run_backward(loss, dev)
    _rel(loss, t["loss"], _tol(dev) / 10)
    for k, p in model.named_parameters():
        if k in t["param_grads"]:
            _rel(p.grad, t["param_grads"][k], 10 * _tol(dev), k)
    model.eval()
    with torch.no_grad():
        for name, fe in (("exact", False), ("faster", True)):
            o, caps_e, ind, ind_aux, _ = _run(model, obj, dev, is_training=False, faster_eval=fe)
            e = g["eval"][name]
            assert torch.equal(caps_e.cpu(), e["captions"]), name
            _rel(o["pred_captions"], e["pred_captions"], _tol(dev), name)
            _rel(torch.stack([x["pred_captions"] for x in o["aux_outputs"]]), e["aux_captions"], _tol(dev), name)
            _indices_equal(ind, e["indices"])


def _check_mm_caption_decoder(golden, dev):
    g = golden("mm_caption_decoder_f64")
    dec = M.multimodal_caption_decoder.MultimodalCaptionDecoder(30, seq_len=8, d_model=64, depth=2, num_heads=4,
                                                                mlp_ratio=4, qkv_bias=True, pre_norm=False,
                                                                return_intermediate=True).double()
    dec = _load(dec, g["state_dict"]).to(dev)
    vm = g["video_memory"].to(dev).requires_grad_(True)
    am = g["audio_memory"].to(dev).requires_grad_(True)
    L = g["tgt"].shape[1]
    look = torch.ones(L, L, dtype=torch.bool, device=dev).triu(1)
    tgt = g["tgt"].to(dev)
    out = dec(tgt=tgt, video_memory=vm, audio_memory=am, tgt_mask=look, tgt_padding_mask=tgt == 1,
              video_memory_padding_mask=g["video_mask"].to(dev), audio_memory_padding_mask=g["audio_mask"].to(dev))
    (out * g["w"].to(dev)).sum().backward()
    _rel(out, g["out"], _tol(dev) / 10)
    _rel(vm.grad, g["grad_video"], _tol(dev))
    _rel(am.grad, g["grad_audio"], _tol(dev))
    for k, p in dec.named_parameters():
        if k in g["param_grads"]:
            _rel(p.grad, g["param_grads"][k], _tol(dev), k)


# --- CPU (oracle MSDA core) -----------------------------------------------------------------------

def test_sparse_dvc_matches_reference_cpu(golden):
    _check_sparse_dvc(golden, "cpu")


def test_deformable_dvc_matches_reference_cpu(golden):
    _check_deformable_dvc(golden, "cpu")


def test_mm_caption_decoder_matches_reference_cpu(golden):
    _check_mm_caption_decoder(golden, "cpu")


def test_state_dict_keys_match_reference(golden):
    for name, build in (("sparse_dvc_f64", build_sparse_dvc), ("deformable_dvc_f64", build_deformable_dvc)):
        ours = {k for k in build().state_dict() if not k.endswith("positional_encoding.pos_embedding")}
        assert ours == set(golden(name)["state_dict"]), name


def _naive_greedy(forward_full, n, length, bos, eos, pad, faster_eval):
    """The reference's decode loop (unimodal_deformable_dvc.py:304-363): full re-decode per word."""
    captions = torch.full((n, length), pad, dtype=torch.int32)
    captions[:, 0] = bos
    done = [False] * n
    for w in range(1, length):
        probs = forward_full(captions)
        tok = probs.argmax(dim=2)
        if faster_eval:
            captions[:, w] = tok[:, w].int()
        else:
            for i in range(n):
                if not done[i]:
                    captions[i, w] = tok[i, w]
                    if tok[i, w] == eos:
                        done[i] = True
    return captions


@pytest.mark.parametrize("kind", ["unimodal", "multimodal"])
@pytest.mark.parametrize("faster_eval", [False, True])
def test_kv_cached_decode_equals_full_redecode(kind, faster_eval):
    torch.manual_seed(5)
    V, d, n, length, K = 40, 32, 4, 9, 15
    bos, eos, pad = 2, 3, 1
    if kind == "unimodal":
        dec = M.unimodal_caption_decoder.UnimodalCaptionDecoder(V, d_model=d, depth=2, num_heads=4, pre_norm=False,
                                                                return_intermediate=True).double().eval()
    else:
        dec = M.multimodal_caption_decoder.MultimodalCaptionDecoder(V, d_model=d, depth=2, num_heads=4, pre_norm=False,
                                                                    return_intermediate=True).double().eval()
    with torch.no_grad():
        dec.head.weight.mul_(8.0)  # confident argmax: no near-ties between the two computations
    mem = torch.randn(n, K, d, dtype=torch.float64)
    mem2 = torch.randn(n, K + 3, d, dtype=torch.float64)
    kmask = torch.zeros(n, K, dtype=torch.bool)
    kmask[1, 9:] = True
    kmask2 = torch.zeros(n, K + 3, dtype=torch.bool)
    kmask2[2, :4] = True
    look = lambda L: torch.ones(L, L, dtype=torch.bool).triu(1)  # noqa: E731
    with torch.no_grad():
        # <eos> takes over the token chosen first for caption 0, so the done bookkeeping is exercised
        first = torch.full((n, length), pad, dtype=torch.int32)
        first[:, 0] = bos
        probe = full_fn(kind, dec, mem, mem2, kmask, kmask2, look, pad)(first)
        tok = int(probe[0, 2].argmax())
        dec.head.weight[eos] = dec.head.weight[tok]
        dec.head.bias[eos] = dec.head.bias[tok] + 0.5
        if kind == "unimodal":
            full = lambda c: dec(c, mem, tgt_mask=look(c.shape[1]), memory_mask=kmask[:, None, None, :],  # noqa: E731
                                 tgt_padding_mask=c == pad)[-1]
            caps, last = dec.greedy_decode(mem, kmask, bos, eos, pad, length, faster_eval)
        else:
            full = lambda c: dec(c, mem, mem2, tgt_mask=look(c.shape[1]), tgt_padding_mask=c == pad,  # noqa: E731
                                 video_memory_padding_mask=kmask, audio_memory_padding_mask=kmask2)[-1]
            caps, last = dec.greedy_decode(mem, kmask, mem2, kmask2, bos, eos, pad, length, faster_eval)
        ref = _naive_greedy(full, n, length, bos, eos, pad, faster_eval)
    assert torch.equal(caps, ref)
    assert (ref == eos).any()


def full_fn(kind, dec, mem, mem2, kmask, kmask2, look, pad):
    if kind == "unimodal":
        return lambda c: dec(c, mem, tgt_mask=look(c.shape[1]), memory_mask=kmask[:, None, None, :],
                             tgt_padding_mask=c == pad)[-1]
    return lambda c: dec(c, mem, mem2, tgt_mask=look(c.shape[1]), tgt_padding_mask=c == pad,
                         video_memory_padding_mask=kmask, audio_memory_padding_mask=kmask2)[-1]


def build_mm_dvc(dev="cpu"):
    a, detr, cap = MG.mm_dvc_args()
    return M.deformable.multimodal_deformable_dvc.MultimodalDeformableDVC(
        ['video', 'audio'], a["num_queries"], a["d_model"], a["num_classes"], True,
        M.matcher.build_matcher(a["matcher"]), 0.5, a["max_eseq_length"], _vocab(), a["seq_len"], None, detr, cap,
        use_differentiable_mask=True).double().to(dev)


def _check_mm_dvc(golden, dev):
    g = golden("mm_dvc_f64")
    model = _load(build_mm_dvc(dev), g["state_dict"])
    obj = _obj_to(g["obj"], dev)
    model.train()
    out, caps, indices, indices_aux, vm, am = _run(model, obj, dev, is_training=True)
    _indices_equal(indices, g["indices"])
    for ours, ref in zip(indices_aux, g["indices_aux"]):
        _indices_equal(ours, ref)
    for k, v in g["out"].items():
        _rel(out[k], v, _tol(dev), k)
    assert torch.equal(caps.cpu(), g["captions"])
    assert torch.equal(vm.cpu(), g["video_mask"]) and torch.equal(am.cpu(), g["audio_mask"])
    _rel(torch.stack([o["pred_captions"] for o in out["aux_outputs"]]), g["aux_captions"], _tol(dev))
    w = {k: v.to(dev) for k, v in g["weights"].items()}
    loss = sum((out[k] * w[k]).sum() for k in w)
    loss = loss + sum((o["pred_captions"] * 0.5).sum() + (o["pred_segments"] * 0.5).sum() for o in out["aux_outputs"])
    _run_backward(loss, dev)
    _rel(loss, g["loss"], _tol(dev) / 10)
    for k, p in model.named_parameters():
        if k in g["param_grads"]:
            _rel(p.grad, g["param_grads"][k], 10 * _tol(dev), k)
    model.eval()
    with torch.no_grad():  # inference (the reference's reads undefined names here): runs, engine.py:71 tuple
        res = _run(model, obj, dev, is_training=False)
    assert len(res) == 6 and res[1].shape == (5, MG.sparse_dvc_args()["seq_len"]) and res[1].dtype == torch.int32


def test_mm_dvc_matches_reference_cpu(golden):
    _check_mm_dvc(golden, "cpu")


# --- GPU (HIP MSDA) -----------------------------------------------------------------------------

@pytest.mark.gpu
def test_sparse_dvc_matches_reference_gpu(golden, dev):
    _check_sparse_dvc(golden, dev)


@pytest.mark.gpu
def test_deformable_dvc_matches_reference_gpu(golden, dev):
    _check_deformable_dvc(golden, dev)


@pytest.mark.gpu
def test_mm_caption_decoder_matches_reference_gpu(golden, dev):
    _check_mm_caption_decoder(golden, dev)


@pytest.mark.gpu
def test_mm_dvc_matches_reference_gpu(golden, dev):
    _check_mm_dvc(golden, dev)


def test_staged_dvc_loss_equals_eager_loss_cpu():
    """StagedDVCLoss (the two-graph DVC step's stages, run eagerly by the trainer) computes
    dvc_workload_loss of the plain forward: fp32 on the CPU with the oracle MSDA core, dropout off."""
    torch.manual_seed(0)
    model = PKG.dvc_core.build_dvc(d_model=64, num_queries=10, T=32, enc_layers=1, dec_layers=2, caption_depth=1,
                                   dropout=0.0, vocab_size=100, ff_dim=128)
    obj = PKG.dvc_core.synthetic_dvc_batch(3, T=32, feature_dim=64, vocab_size=100, seed=3)
    with oracle_core(PKG):
        loss_e = PKG.dvc_core.dvc_workload_loss(model(obj, is_training=True), obj)
        sl = PKG.dvc_core.StagedDVCLoss(obj, model)
        tr = PKG.train_step.FlatGradTrainer(model, sl, lr=1e-3, use_bf16=False, graph=False)
        assert tr.staged
        loss_s = tr._forward_backward((obj,))
    torch.testing.assert_close(loss_s, loss_e.detach(), rtol=1e-6, atol=1e-6)
    assert torch.isfinite(tr.flat_grad).all() and tr.flat_grad.abs().sum() > 0


def test_level_terms_equal_per_level_loop_cpu():
    """dvc_core.level_terms (every decoder level's loss terms in one launch each, from the heads and
    caption probabilities stacked over the levels, ``out['_levels']``) equals the per-level loop of
    dvc_workload_loss on the same forward result, value and gradients (fp32, CPU, oracle MSDA core)."""
    torch.manual_seed(1)
    model = PKG.dvc_core.build_dvc(d_model=64, num_queries=10, T=32, enc_layers=1, dec_layers=3, caption_depth=1,
                                   dropout=0.0, vocab_size=100, ff_dim=128)
    obj = PKG.dvc_core.synthetic_dvc_batch(3, T=32, feature_dim=64, vocab_size=100, seed=5)
    grads = []
    with oracle_core(PKG):
        for vectorized in (True, False):
            model.zero_grad(set_to_none=True)
            res = model(obj, is_training=True)
            assert '_levels' in res[0] and res[0]['_levels']['segments'].shape[0] == 3
            if not vectorized:
                res[0].pop('_levels')
            loss = PKG.dvc_core.dvc_workload_loss(res, obj)
            loss.backward()
            grads.append((loss.detach(), [p.grad.clone() for p in model.parameters() if p.grad is not None]))
    (l1, g1), (l2, g2) = grads
    torch.testing.assert_close(l1, l2, rtol=1e-6, atol=1e-6)
    assert len(g1) == len(g2) > 0
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("faster_eval", [False, True])
def test_oracle_redecode_loop_matches_kv_cached_decode(faster_eval):
    """bench.py --config decode's CPU leg decodes with oracle/cpu_model.redecode_greedy (the
    reference's full re-decode per word, unimodal_deformable_dvc.py:318-354): the same captions as
    the KV-cached greedy_decode, and the same input for the final word's pass."""
    from oracle.cpu_model import redecode_greedy
    torch.manual_seed(6)
    V, d, n, length, K = 40, 32, 4, 9, 15
    dec = M.unimodal_caption_decoder.UnimodalCaptionDecoder(V, d_model=d, depth=2, num_heads=4, pre_norm=False,
                                                            return_intermediate=True).double().eval()
    with torch.no_grad():
        dec.head.weight.mul_(8.0)
        mem = torch.randn(n, K, d, dtype=torch.float64)
        kmask = torch.zeros(n, K, dtype=torch.bool)
        kmask[2, 7:] = True
        caps, last = dec.greedy_decode(mem, kmask, 2, 3, 1, length, faster_eval)
        caps_r, last_r = redecode_greedy(dec, mem, kmask, 2, 3, 1, length, faster_eval)
    assert torch.equal(caps, caps_r) and torch.equal(last, last_r)
