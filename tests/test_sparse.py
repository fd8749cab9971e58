"""Sparse-DETR transformer mirror (models/sparse/unimodal_sparse_deformable_transformer.py)
against the reference's own run (tests/golden/sparse_f64.pt: rho = 0.3, mask predictor,
top-k encoder queries over the full pyramid scattered back, 2 enc + 2 dec layers, fp64).

CPU: the module logic with the MSDA core replaced by the oracle (oracle/cpu_model.oracle_core).
GPU: the same on the HIP kernels (MSDA fwd/bwd with Lq = top-k, fused prologue), plus the
decoder attention map of its own sampling locations through the DAM kernel.
Tolerance: fp64; the reference's sine/cos position terms are not involved here, so 1e-9."""
import pytest
import torch

from conftest import PKG

SP = PKG.models.sparse.unimodal_sparse_deformable_transformer


def _build(g, device):
    torch.manual_seed(0)
    tr = SP.SparseDeformableTransformer(d_model=64, num_head=4, num_encoder_layers=2, num_decoder_layers=2,
                                        dim_feedforward=128, dropout=0.0, return_intermediate_dec=True,
                                        num_feature_levels=4, dec_n_points=4, enc_n_points=4, rho=0.3).double()
    tr.load_state_dict({k: v.double() for k, v in g["state_dicts"]["transformer"].items()})
    qe = torch.nn.Embedding(12, 128).double()
    qe.load_state_dict({k: v.double() for k, v in g["state_dicts"]["query_embedding"].items()})
    return tr.to(device), qe.to(device)


def _run(g, device):
    tr, qe = _build(g, device)
    srcs = [s.to(device).requires_grad_(True) for s in g["srcs"]]
    pos = [p.to(device) for p in g["pos"]]
    masks = [m.to(device) for m in g["masks"]]
    (src_flatten, shapes, starts, valid, lvl_pos, mask_flatten, proposals, topk, mask_pred,
     sparse_token_nums) = tr.prepare_encoder_inputs(srcs, masks, pos)
    memory, sl_enc, aw_enc, _, _ = tr.forward_encoder(src_flatten, shapes, starts, valid, lvl_pos, mask_flatten,
                                                      proposals, topk, sparse_token_nums)
    B = srcs[0].shape[0]
    qmask = torch.ones(B, 12, dtype=torch.bool, device=device)
    _, tgt, refp, qpos = tr.prepare_decoder_input_query(B, qe.weight)
    hs, inter, sl_dec, aw_dec = tr.forward_decoder(tgt, refp, memory, shapes, starts, valid, qpos, mask_flatten,
                                                   qmask, False)
    w = [t.to(device) for t in g["weights"]]
    ((hs * w[0]).sum() + (memory * w[1]).sum() + (mask_pred * w[2]).sum()).backward()
    return dict(tr=tr, qe=qe, srcs=srcs, hs=hs, memory=memory, mask_pred=mask_pred, topk=topk,
                sparse_token_nums=sparse_token_nums, sl_enc=sl_enc, aw_enc=aw_enc, sl_dec=sl_dec, aw_dec=aw_dec,
                shapes=shapes, starts=starts)


def _check(r, g, tol):
    def close(a, b):
        torch.testing.assert_close(a.detach().cpu().to(b.dtype), b, rtol=tol, atol=tol)
    assert torch.equal(r["topk"].cpu(), g["topk"])
    assert torch.equal(r["sparse_token_nums"].cpu(), g["sparse_token_nums"])
    close(r["mask_pred"], g["mask_prediction"])
    close(r["memory"], g["memory"])
    close(r["hs"], g["hs"])
    close(r["sl_enc"], g["sampling_locations_enc"])
    close(r["aw_enc"], g["attn_weights_enc"])
    close(r["sl_dec"], g["sampling_locations_dec"])
    close(r["aw_dec"], g["attn_weights_dec"])
    for s, ref in zip(r["srcs"], g["grad_srcs"]):
        close(s.grad, ref)
    for k, p in r["tr"].named_parameters():
        if k in g["param_grads"]["transformer"]:
            torch.testing.assert_close(p.grad.detach().cpu(), g["param_grads"]["transformer"][k], rtol=tol * 10,
                                       atol=tol * 10, msg=k)


def test_sparse_transformer_matches_reference_cpu(golden):
    from oracle.cpu_model import oracle_core
    g = golden("sparse_f64")
    with oracle_core(PKG):
        r = _run(g, "cpu")
    _check(r, g, 1e-9)


@pytest.mark.gpu
def test_sparse_transformer_matches_reference_gpu(golden, dev):
    g = golden("sparse_f64")
    r = _run(g, dev)
    _check(r, g, 1e-9)
    # the criterion's decoder attention map of the model's own sampling locations (DAM kernel)
    dam = PKG.utils.dam.attn_map_to_flat_grid(r["shapes"], r["starts"], r["sl_dec"].detach(), r["aw_dec"].detach())
    ref = g["dam_flat_grid"]
    torch.testing.assert_close(dam.cpu(), ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())


@pytest.mark.gpu
def test_static_topk_width_matches_data_dependent_width(dev):
    """SparseDVCCore's top-k width from the shapes (min(S, int(S*rho)+1), no device read) selects
    the same encoder tokens per clip as the reference's max(sparse_token_nums) width (:212) — the
    per-clip keep masks cut both to each clip's count — on padded clips: identical outputs (every MSDA
    query is computed independently, so the extra masked-out queries change nothing)."""
    import copy
    torch.manual_seed(0)
    core = PKG.dvc_core.SparseDVCCore(d_model=64, num_queries=6, feature_dim=64, enc_layers=2, dec_layers=2,
                                      ff_dim=128, dropout=0.0).to(dev)
    ref_core = copy.deepcopy(core)
    ref_core.unimodal_sparse_transformer.static_topk = False
    video, mask, dur = PKG.dvc_core.synthetic_clips(3, T=64, feature_dim=64, padded=True, seed=5, device=dev)
    a, b = core(video, mask, dur), ref_core(video, mask, dur)
    assert a["sparse_topk"] >= b["sparse_topk"]
    for k in ("hs", "memory", "all_segments", "all_counts"):
        torch.testing.assert_close(a[k], b[k], rtol=0, atol=0, msg=k)
    torch.testing.assert_close(PKG.dvc_core.sparse_workload_loss(a), PKG.dvc_core.sparse_workload_loss(b),
                               rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_sparse_step_is_graph_captured(dev):
    """With the static top-k width the Sparse-DETR training step has no host read and is replayed
    as HIP graphs; replays track the eager step."""
    import copy
    torch.manual_seed(0)
    base = PKG.dvc_core.SparseDVCCore(d_model=64, num_queries=6, feature_dim=64, enc_layers=1, dec_layers=1,
                                      ff_dim=128, dropout=0.0)
    batch = PKG.dvc_core.synthetic_clips(2, T=64, feature_dim=64, padded=False, seed=3, device=dev)
    mk = lambda g: PKG.train_step.FlatGradTrainer(copy.deepcopy(base).to(dev), PKG.dvc_core.sparse_workload_loss,  # noqa
                                                  lr=1e-4, use_bf16=True, graph=g)
    tg, te = mk(True), mk(False)
    tg.capture(batch, warmup=2)
    for _ in range(2):
        te.step(batch)
    for _ in range(3):
        lg, le = tg.step(batch).item(), te.step(batch).item()
        assert abs(lg - le) <= 1e-2 * abs(le) + 1e-2


@pytest.mark.gpu
def test_sparse_encoder_carry_matches_plain_bf16(dev, monkeypatch):
    """Under bf16 autocast the Sparse-DETR encoder carries its 16-bit operands between layers
    (``DeformableTransformerEncoderLayer.forward_carry``: bf16(tgt + pos) and bf16(tgt) from the
    fused add + LayerNorm, the whole memory's bf16 copy kept up to date by the same scatter as the
    fp32 memory).  Against the plain layer path (MFL_SPARSE_CARRY=0) on padded clips (per-clip
    top-k counts: the keep masks): the forward is the same arithmetic, bit for bit.  Gradients are
    the same terms summed in another order (fp32), so each is held to the fp64 run of the same model:
    within 2e-3 relative of the plain path's gradient, or — for a gradient whose sum cancels (the
    BaseEncoder's biases: a sum over every token) — no further from the fp64 gradient than 1.5x the
    plain path's own distance + 2e-3."""
    import copy
    torch.manual_seed(0)
    core = PKG.dvc_core.SparseDVCCore(d_model=256, num_queries=10, feature_dim=256, num_heads=4, enc_layers=3,
                                      dec_layers=2, ff_dim=512, dropout=0.0).to(dev)
    video, mask, dur = PKG.dvc_core.synthetic_clips(3, T=128, feature_dim=256, padded=True, seed=7, device=dev)
    res = []
    # carry with the row write-backs (_ScatterRows: the fp32 memory written once), carry with the
    # per-layer scatters, the plain layer path
    for carry, rows_ in (("1", "1"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("MFL_SPARSE_CARRY", carry)
        monkeypatch.setenv("MFL_SPARSE_ROWS", rows_)
        core.zero_grad(set_to_none=True)
        PKG._trace.clear()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = core(video, mask, dur)
            loss = PKG.dvc_core.sparse_workload_loss(out)
        loss.backward()
        assert (PKG._trace.hits.get("sparse_rows", 0) > 0) == (carry == "1" and rows_ == "1")
        res.append(([out[k].detach().float().clone() for k in ("memory", "hs", "all_segments", "all_counts")],
                    {n: p.grad.detach().clone() for n, p in core.named_parameters() if p.grad is not None}))
    (fr, gr) = res.pop(0)
    for x, y in zip(fr, res[0][0]):
        assert torch.equal(x, y)
    core64 = copy.deepcopy(core).double()
    core64.zero_grad(set_to_none=True)
    torch.set_default_dtype(torch.float64)  # (tensors the model allocates with the default dtype)
    try:
        PKG.dvc_core.sparse_workload_loss(core64(video.double(), mask, dur.double())).backward()
    finally:
        torch.set_default_dtype(torch.float32)
    g64 = {n: p.grad.detach() for n, p in core64.named_parameters() if p.grad is not None}
    (fa, ga), (fb, gb) = res
    for x, y in zip(fa, fb):
        assert torch.equal(x, y)
    assert ga.keys() == gb.keys() == gr.keys() and len(ga) > 20

    def rel(a, b):
        return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()

    rows, bad = [], []
    for n in ga:
        for gx in (ga, gr):  # (both carry paths against the plain one)
            d_ab = rel(gx[n], gb[n])
            e_a, e_b = rel(gx[n], g64[n]), rel(gb[n], g64[n])
            rows.append((n, round(d_ab, 5), round(e_a, 5), round(e_b, 5)))
            if d_ab >= 2e-3 and e_a > 1.5 * e_b + 2e-3:
                bad.append(rows[-1])
    print("carry vs plain (name, difference, carry vs fp64, plain vs fp64), largest:",
          sorted(rows, key=lambda r: -r[1])[:6])
    assert not bad, bad
