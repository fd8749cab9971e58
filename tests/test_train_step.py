"""The bench's training step (train_step.FlatGradTrainer): flat-gradient fwd+bwd, gradient
all-reduce, clip_grad_norm_ + AdamW.

CPU (no marker): the eager step equals the textbook PyTorch step (model.backward, clip,
AdamW), and the world_size-2 gloo run — each rank one clip, one flat all-reduce — equals the
single-process step on both clips, i.e. the reference's DDP semantics (gradients averaged
over ranks, main.py:55,98).  The MSDA core runs through the oracle on the CPU.
GPU (-m gpu): the HIP-graph replay of the step equals the eager step.
"""
import copy
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

SMALL = dict(d_model=64, num_queries=6, feature_dim=64, enc_layers=1, dec_layers=1, ff_dim=128, dropout=0.0,
             num_classes=5)


def _model(device="cpu"):
    torch.manual_seed(0)
    return PKG.dvc_core.DeformableDVCCore(**SMALL).to(device)


def _batch(n, device="cpu"):
    return PKG.dvc_core.synthetic_clips(n, T=32, feature_dim=64, padded=True, seed=3, device=device)


def _params(model):
    return {k: v.detach().clone().cpu() for k, v in model.named_parameters()}


def test_eager_step_matches_textbook_step():
    from oracle.cpu_model import oracle_core
    batch = _batch(2)
    ref = _model()
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=1e-4)
    mine = copy.deepcopy(ref)
    tr = PKG.train_step.FlatGradTrainer(mine, PKG.dvc_core.workload_loss, lr=1e-3, weight_decay=1e-4,
                                        max_norm=0.1, use_bf16=False, graph=False)
    with oracle_core(PKG):
        for _ in range(2):
            PKG.dvc_core.workload_loss(ref(*batch)).backward()
            torch.nn.utils.clip_grad_norm_(ref.parameters(), 0.1)
            opt.step()
            opt.zero_grad(set_to_none=True)
            tr.eager_step(batch)
    a, b = _params(ref), _params(mine)
    for k in a:
        torch.testing.assert_close(b[k], a[k], rtol=1e-5, atol=1e-6, msg=k)
    # every parameter got a gradient view into the single flat buffer
    assert all(p.grad.data_ptr() >= tr.flat_grad.data_ptr() for p in tr.params)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    import importlib
    pkg = importlib.import_module("multimodal-feature-learning_amd")
    from oracle.cpu_model import oracle_core
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        model = pkg.dvc_core.DeformableDVCCore(**SMALL)
        video, mask, dur = pkg.dvc_core.synthetic_clips(2, T=32, feature_dim=64, padded=True, seed=3)
        shard = (video[rank:rank + 1], mask[rank:rank + 1], dur[rank:rank + 1])
        # small buckets: several all-reduces overlapped with the backward
        tr = pkg.train_step.FlatGradTrainer(model, pkg.dvc_core.workload_loss, lr=1e-3, weight_decay=1e-4,
                                            max_norm=0.1, use_bf16=False, graph=False, bucket_mb=0.05)
        assert tr.world == world and tr.overlap and len(tr.buckets) > 3
        with oracle_core(pkg):
            tr._forward_backward(shard)
            tr._allreduce()
            grad = tr.flat_grad.clone()
            tr._update()
            tr.eager_step(shard)
        torch.save({"grad": grad, "params": {k: v.detach() for k, v in model.named_parameters()}},
                   f"{out_path}.{rank}")
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_equal_full_batch_step():
    """Each rank one clip; after the flat all-reduce every rank holds the gradient of the
    two-clip batch averaged over ranks (compared before AdamW, whose sign-like first steps
    would amplify fp32 summation-order noise), and the ranks' parameters stay identical."""
    from oracle.cpu_model import oracle_core
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "params")
        mp.start_processes(_rank_main, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
        r0 = torch.load(out + ".0", weights_only=True)
        r1 = torch.load(out + ".1", weights_only=True)
    ref = _model()
    tr = PKG.train_step.FlatGradTrainer(ref, lambda o: PKG.dvc_core.workload_loss(o) / 2, lr=1e-3,
                                        weight_decay=1e-4, max_norm=0.1, use_bf16=False, graph=False)
    with oracle_core(PKG):
        tr._forward_backward(_batch(2))
    full = tr.flat_grad
    assert torch.equal(r0["grad"], r1["grad"])
    err = (r0["grad"] - full).abs().max().item()
    assert err <= 1e-5 * full.abs().max().item(), (err, full.abs().max().item())
    for k in r0["params"]:
        assert torch.equal(r0["params"][k], r1["params"][k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("bf16", [False, True])
def test_graph_replay_matches_eager_step(dev, bf16):
    """The captured fwd+bwd graph produces the eager step's loss and flat gradient on the
    same parameters; the update graph then applies clip + AdamW like the eager update."""
    batch = _batch(2, dev)
    model = _model(dev)
    tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.workload_loss, lr=1e-3, max_norm=0.1, use_bf16=bf16,
                                        graph=True)
    tr.capture(batch, warmup=1)
    tr._g_fb.replay()
    loss_g, grad_g = tr._loss.clone(), tr.flat_grad.clone()
    loss_e = tr._forward_backward(batch)
    grad_e = tr.flat_grad.clone()
    torch.cuda.synchronize()
    torch.testing.assert_close(loss_g, loss_e, rtol=1e-5, atol=1e-5)
    err = (grad_g - grad_e).abs().max().item()
    assert err <= 1e-4 * grad_e.abs().max().item(), (err, grad_e.abs().max().item())
    before = _params(model)
    tr._g_up.replay()
    torch.cuda.synchronize()
    after = _params(model)
    assert any(not torch.equal(before[k], after[k]) for k in before)
    assert all(torch.isfinite(v).all() for v in after.values())


@pytest.mark.gpu
def test_graph_steps_track_eager_steps_at_bench_shape(dev):
    """Five graph-replayed steps at the bench shape (configs[1], bf16) follow five eager steps
    from the same initial weights, with allocating device work (norms, maxima) between the
    replays.  With the HIP runtime's graph packet capture on, this sequence corrupted the
    second replay's gradients (inf / NaN); the package turns it off (__init__.py)."""
    assert os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "0"
    torch.manual_seed(0)
    base = PKG.dvc_core.DeformableDVCCore(d_model=512, num_queries=100, dropout=0.0)
    batch = PKG.dvc_core.synthetic_clips(8, T=1024, seed=1000, device=dev)
    mk = lambda graph: PKG.train_step.FlatGradTrainer(  # noqa: E731
        copy.deepcopy(base).to(dev), PKG.dvc_core.workload_loss, lr=1e-4, weight_decay=1e-4, max_norm=0.1,
        use_bf16=True, graph=graph)
    tg, te = mk(True), mk(False)
    tg.capture(batch)
    for _ in range(3):  # capture() ran three eager warm-up steps: same starting point
        te.step(batch)
    for i in range(5):
        lg = tg.step(batch).item()
        gnorm_g = tg.flat_grad.norm().item()  # allocating eager work between replays
        assert bool(torch.isfinite(tg.flat_param).all()) and gnorm_g == gnorm_g, i
        le = te.step(batch).item()
        gnorm_e = te.flat_grad.norm().item()
        assert abs(lg - le) <= 1e-2 * abs(le) + 1.0, (i, lg, le)
        assert abs(gnorm_g - gnorm_e) <= 1e-2 * gnorm_e, (i, gnorm_g, gnorm_e)


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["multimodal", "sparse"])
def test_other_dvc_cores_train_one_step(config):
    """configs[2] (video + audio) and the Sparse-DETR DVC: one bf16 training step through the
    trainer is finite and moves every parameter that receives a gradient."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    small = dict(d_model=64, num_queries=6, feature_dim=64, enc_layers=1, dec_layers=2, ff_dim=128, dropout=0.0)
    video, vmask, dur = PKG.dvc_core.synthetic_clips(2, T=64, feature_dim=64, padded=True, device=dev)
    if config == "multimodal":
        model = PKG.dvc_core.MultimodalDVCCore(num_classes=5, **small).to(dev)
        audio, amask, _ = PKG.dvc_core.synthetic_clips(2, T=16, feature_dim=64, padded=True, seed=9, device=dev)
        batch, loss_fn = (video, vmask, audio, amask, dur), PKG.dvc_core.multimodal_workload_loss
    else:
        model = PKG.dvc_core.SparseDVCCore(**small).to(dev)
        batch, loss_fn = (video, vmask, dur), PKG.dvc_core.sparse_workload_loss
    before = {k: v.detach().clone() for k, v in model.named_parameters()}
    tr = PKG.train_step.FlatGradTrainer(model, loss_fn, lr=1e-3, use_bf16=True, graph=False)
    loss = tr.eager_step(batch)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item()
    assert torch.isfinite(tr.flat_grad).all().item() and tr.flat_grad.abs().sum().item() > 0
    moved = sum(int(not torch.equal(before[k], v.detach())) for k, v in model.named_parameters())
    assert moved > len(before) // 2


@pytest.mark.gpu
def test_fused_flat_adamw_matches_torch_adamw():
    """csrc/flat_adamw.hip (clip_grad_norm_ + AdamW over the flat buffers, bf16 shadow in the
    same pass) against torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW on the same model,
    fp32, three steps with the clip active (max_norm 0.1) and inactive (max_norm 1e6).
    Tolerance: fp32 (the two order their norm sums differently)."""
    dev = torch.device("cuda", 0)
    batch = _batch(2, dev)
    for max_norm in (0.1, 1e6):
        ref, mine = _model(dev), _model(dev)
        t_ref = PKG.train_step.FlatGradTrainer(ref, PKG.dvc_core.workload_loss, lr=1e-3, weight_decay=1e-2,
                                               max_norm=max_norm, use_bf16=False, graph=False, fused_optimizer=False)
        t_mine = PKG.train_step.FlatGradTrainer(mine, PKG.dvc_core.workload_loss, lr=1e-3, weight_decay=1e-2,
                                                max_norm=max_norm, use_bf16=False, graph=False, fused_optimizer=True)
        for _ in range(3):  # the same gradients into both optimizers (the MSDA backward's LDS-atomic
            t_ref._forward_backward(batch)  # list order would otherwise flip Adam's sign on ~0 grads)
            t_mine.flat_grad.copy_(t_ref.flat_grad)
            t_ref._update()
            t_mine._update()
        torch.cuda.synchronize()
        torch.testing.assert_close(t_mine.flat_param, t_ref.flat_param, rtol=2e-5, atol=2e-6)
        assert float(t_mine.opt_step.item()) == 3.0
    # bf16 trainer: the shadow written by the optimizer pass is exactly the cast of the new weights
    m = _model(dev)
    t = PKG.train_step.FlatGradTrainer(m, PKG.dvc_core.workload_loss, lr=1e-3, use_bf16=True, graph=False)
    t.eager_step(batch)
    torch.cuda.synchronize()
    assert torch.equal(t.flat_bf16, t.flat_param.to(torch.bfloat16))


def test_capture_refuses_when_graph_packet_capture_is_on():
    """capture() raises unless the HIP runtime's graph packet capture is off; checked
    before any device work, so it runs on the CPU (fresh process: the variable is read at import)."""
    import subprocess
    import sys
    code = (
        "import sys, importlib; sys.path.insert(0, %r)\n"
        "pkg = importlib.import_module('multimodal-feature-learning_amd')\n"
        "assert not pkg.graph_packet_capture_off()\n"
        "import torch\n"
        "torch.manual_seed(0)\n"
        "m = pkg.dvc_core.DeformableDVCCore(d_model=64, num_queries=6, feature_dim=64, enc_layers=1, dec_layers=1,"
        " ff_dim=128, dropout=0.0)\n"
        "tr = pkg.train_step.FlatGradTrainer(m, pkg.dvc_core.workload_loss, use_bf16=False, graph=True)\n"
        "try:\n"
        "    tr.capture(None)\n"
        "except RuntimeError as e:\n"
        "    assert 'DEBUG_CLR_GRAPH_PACKET_CAPTURE' in str(e)\n"
        "    print('refused')\n"
    ) % ROOT
    env = dict(os.environ, DEBUG_CLR_GRAPH_PACKET_CAPTURE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "refused" in r.stdout, r.stderr


@pytest.mark.gpu
def test_learning_rate_change_reaches_the_replayed_update(dev):
    """lr lives in device memory read by the update kernels: a schedule step between replays
    (reference main.py:99 StepLR) changes what the captured update graph does."""
    batch = _batch(2, dev)
    model = _model(dev)
    tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.workload_loss, lr=1e-3, weight_decay=1e-2,
                                        max_norm=0.1, use_bf16=True, graph=True)
    tr.capture(batch, warmup=1)
    tr._g_fb.replay()
    tr.lr = 0.0  # no step and no decay (1 - lr * wd = 1)
    before = tr.flat_param.clone()
    tr._g_up.replay()
    torch.cuda.synchronize()
    assert torch.equal(tr.flat_param, before)
    tr.lr = 1e-3
    tr._g_up.replay()
    torch.cuda.synchronize()
    assert not torch.equal(tr.flat_param, before)


@pytest.mark.gpu
def test_dropout_masks_are_fresh_on_every_replay(dev):
    """The fused dropout kernels draw their keep bits from a device seed made by torch.randint
    inside the captured graph: two replays on the same weights and inputs give different
    gradients (a seed frozen at capture would replay the same masks every step)."""
    torch.manual_seed(0)
    model = PKG.dvc_core.DeformableDVCCore(**dict(SMALL, dropout=0.1)).to(dev)
    batch = _batch(2, dev)
    tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.workload_loss, lr=1e-3, use_bf16=True, graph=True)
    tr.capture(batch, warmup=1)
    tr._g_fb.replay()
    g1 = tr.flat_grad.clone()
    tr._g_fb.replay()
    g2 = tr.flat_grad.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(g1).all() and torch.isfinite(g2).all()
    assert not torch.equal(g1, g2)


@pytest.mark.parametrize("bucket_mb", [0.001, 0.05, 32.0])
def test_buckets_cover_every_parameter_once_in_reverse_order(bucket_mb):
    """The all-reduce buckets: contiguous ranges of the flat buffer that tile it exactly, every
    parameter in exactly one bucket, the last parameters (the backward's first gradients) first."""
    model = _model()
    tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.workload_loss, use_bf16=False, graph=False,
                                        bucket_mb=bucket_mb)
    seen = sorted(i for _, _, idx in tr.buckets for i in idx)
    assert seen == list(range(len(tr.params)))
    ends = [(s, e) for s, e, _ in tr.buckets]
    assert ends[0][1] == tr.flat_grad.numel() and ends[-1][0] == 0
    for (s0, _), (_, e1) in zip(ends, ends[1:]):
        assert e1 == s0  # reverse order, no gap, no overlap
    cap = int(bucket_mb * 2 ** 20 / 4)
    for s_, e, idx in tr.buckets:
        assert e - s_ == sum((tr.params[i].numel() + 3) // 4 * 4 for i in idx)  # 16-B aligned spans
        assert e - s_ <= cap or len(idx) == 1


def _nccl_rank_main(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    import importlib
    pkg = importlib.import_module("multimodal-feature-learning_amd")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        base = pkg.dvc_core.DeformableDVCCore(**SMALL)
        batch = pkg.dvc_core.synthetic_clips(2, T=32, feature_dim=64, padded=True, seed=3, device=dev)
        res = {}
        for name, kw in (("plain", dict(overlap=False)), ("overlap", dict(overlap="force", bucket_mb=0.05))):
            tr = pkg.train_step.FlatGradTrainer(copy.deepcopy(base).to(dev), pkg.dvc_core.workload_loss, lr=1e-3,
                                                use_bf16=False, graph=False, **kw)
            tr._forward_backward(batch)
            tr._allreduce()
            res[name] = tr.flat_grad.cpu()
        # graph mode: the bucket all-reduces captured with the backward
        tr = pkg.train_step.FlatGradTrainer(copy.deepcopy(base).to(dev), pkg.dvc_core.workload_loss, lr=1e-3,
                                            use_bf16=False, graph=True, overlap="force", bucket_mb=0.05)
        assert tr.capture_collectives
        tr.capture(batch, warmup=1)
        tr._g_fb.replay()
        torch.cuda.synchronize()
        res["graph"] = tr.flat_grad.cpu()
        res["graph_reduces"] = tr._fb_reduces
        tr._forward_backward(batch)  # eager, same weights (the warm-up step moved them)
        torch.cuda.synchronize()
        res["graph_eager"] = tr.flat_grad.cpu()
        torch.save(res, out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_one_rank_bucketed_allreduce_smoke(dev):
    """The RCCL code path on one GPU: an nccl (= RCCL) process group of world size 1, the bucket
    all-reduces overlapped with the backward (forced at one rank) eagerly and captured in the
    fwd+bwd graph, against the trainer without collectives (one rank: the all-reduce is identity)."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "nccl.pt")
        mp.start_processes(_nccl_rank_main, args=(1, _free_port(), out), nprocs=1, join=True, start_method="spawn")
        r = torch.load(out, weights_only=True)
    torch.testing.assert_close(r["overlap"], r["plain"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(r["graph"], r["graph_eager"], rtol=1e-4, atol=1e-5)
    assert r["graph_reduces"]


def test_parameters_without_gradients_are_left_untouched():
    """MultimodalDVCCore has parameters the forward never uses (pos_trans / pos_trans_norm, as the
    reference's multimodal transformer): the reference's AdamW skips them (grad None, DDP
    find_unused_parameters); the trainer leaves their values alone as well — no weight decay."""
    from oracle.cpu_model import oracle_core
    torch.manual_seed(0)
    model = PKG.dvc_core.MultimodalDVCCore(**{k: v for k, v in SMALL.items() if k != "num_classes"})
    v = PKG.dvc_core.synthetic_clips(1, T=32, feature_dim=64, seed=1)
    a = PKG.dvc_core.synthetic_clips(1, T=16, feature_dim=64, seed=2)
    before = _params(model)
    tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.multimodal_workload_loss, lr=1e-2, weight_decay=0.5,
                                        use_bf16=False, graph=False)
    with oracle_core(PKG):
        for _ in range(2):
            tr.eager_step((v[0], v[1], a[0], a[1], v[2]))
    after = _params(model)
    unused = [k for k in before if "pos_trans" in k]
    assert unused and len(tr._unused) == len(unused)
    for k in unused:
        torch.testing.assert_close(after[k], before[k], rtol=0, atol=0, msg=k)
    assert any(not torch.equal(after[k], before[k]) for k in before if k not in unused)


@pytest.mark.gpu
def test_fused_update_leaves_unused_parameters_untouched(dev):
    torch.manual_seed(0)
    model = PKG.dvc_core.MultimodalDVCCore(**{k: v for k, v in SMALL.items() if k != "num_classes"}).to(dev)
    v = PKG.dvc_core.synthetic_clips(2, T=32, feature_dim=64, seed=1, device=dev)
    a = PKG.dvc_core.synthetic_clips(2, T=16, feature_dim=64, seed=2, device=dev)
    before = _params(model)
    tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.multimodal_workload_loss, lr=1e-2, weight_decay=0.5,
                                        use_bf16=True, graph=True)
    batch = (v[0], v[1], a[0], a[1], v[2])
    tr.capture(batch, warmup=2)
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    after = _params(model)
    unused = [k for k in before if "pos_trans" in k]
    assert unused
    for k in unused:
        torch.testing.assert_close(after[k], before[k], rtol=0, atol=0, msg=k)


def test_flat_order_lays_query_projection_pairs_back_to_back():
    """FlatGradTrainer's flat layout puts each MSDeformAttn's sampling_offsets / attention_weights
    weights (and biases) next to each other (MSDeformAttn.flat_groups), keeping every parameter
    once: the fused query projection then reads [W_off; W_aw] as one view of the bf16 shadow."""
    model = _model()
    tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.workload_loss, use_bf16=False, graph=False)
    assert sorted(map(id, tr.params)) == sorted(id(p) for p in model.parameters() if p.requires_grad)
    pos = {id(p): i for i, p in enumerate(tr.params)}
    att = [m for m in model.modules() if isinstance(m, PKG.models.modules.attention.MSDeformAttn)]
    assert att
    for m in att:
        for a, b in m.flat_groups():
            assert pos[id(b)] == pos[id(a)] + 1
            assert b.data_ptr() == a.data_ptr() + a.numel() * a.element_size()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["multimodal", "sparse"])
def test_grad_sum_in_gemm(dev, monkeypatch, kind):
    """linear.mark_grad_sum: an activation whose every consumer takes part (configs[2]'s encoder: the
    joint rows' bf16 self-block output is the cross-modal calls' value and their query, the FFN input
    linear1's input and the residual; the Sparse-DETR encoder: the bf16 memory copy is the next layer's MSDA value
    and its row write-back's input) gets its input gradients summed in the later consumer's dgrad
    GEMM (C += dY W) instead of autograd's bf16 add.  Same loss; the flat gradient differs from
    autograd's sums only by that one bf16 rounding per summed pair."""
    # (d_model 256: the fused carry paths, which tag the activations, need d % 256 == 0)
    small = dict(d_model=256, num_queries=6, feature_dim=256, num_heads=4, enc_layers=2, dec_layers=2, ff_dim=512,
                 dropout=0.0)
    if kind == "multimodal":
        video, vmask, dur = PKG.dvc_core.synthetic_clips(2, T=256, feature_dim=256, padded=True, device=dev)
        audio, amask, _ = PKG.dvc_core.synthetic_clips(2, T=16, feature_dim=256, padded=True, seed=9, device=dev)
        batch = (video, vmask, audio, amask, dur)
        make = lambda: PKG.dvc_core.MultimodalDVCCore(num_classes=5, **small)  # noqa: E731
        # encoder: 2 layers x (the joint rows' bf16 self-block output x16 — both cross calls' value and
        # query — and the joint FFN input; _forward_joint); decoder: 2 layers x (the one bf16 query of
        # both cross-attentions, the bridge output t: linear1's input and the residual)
        loss_fn, want = PKG.dvc_core.multimodal_workload_loss, 8
    else:
        batch = PKG.dvc_core.synthetic_clips(3, T=128, feature_dim=256, padded=True, seed=7, device=dev)
        make = lambda: PKG.dvc_core.SparseDVCCore(**small)  # noqa: E731
        loss_fn, want = PKG.dvc_core.sparse_workload_loss, 2  # the bf16 memory copy before each layer

    def run(on):
        monkeypatch.setattr(PKG.models.modules.linear, "GRAD_SUM_IN_GEMM", on)
        torch.manual_seed(0)
        tr = PKG.train_step.FlatGradTrainer(make().to(dev), loss_fn, lr=1e-3, use_bf16=True, graph=False)
        PKG._trace.clear()
        loss = tr._forward_backward(batch)
        torch.cuda.synchronize()
        return loss, tr.flat_grad.clone(), dict(PKG._trace.hits), [p.numel() for p in tr.params], tr._offs

    loss_r, ref, hits_r, sizes, offs = run(False)
    loss, got, hits, _, _ = run(True)
    assert hits_r.get("grad_sum_into", 0) == 0 and hits.get("grad_sum_into", 0) == want, hits
    assert torch.equal(loss, loss_r)
    assert ((got - ref).norm() / ref.norm()).item() < 5e-3
    for i, (n, off) in enumerate(zip(sizes, offs)):
        a, b = got[off:off + n].double(), ref[off:off + n].double()
        assert (a - b).norm().item() <= 2e-2 * b.norm().item() + 1e-6, i


@pytest.mark.gpu
def test_shared_layer_gradients_accumulate_into_flat_views(dev, monkeypatch):
    """configs[2]'s encoder calls one self-attention module four times a layer (the two video calls
    take the weight-gradient GEMMs, the two short audio ones the deferred queue) and its decoder one
    cross-attention twice: in the trainer a later call adds its weight / bias products into the flat
    view an earlier call handed to autograd (linear._accum_target / _accum_group), and the queue adds
    its batched products into .grad in place (the trainer's _accum_target).  The flat gradient is the
    one autograd's own accumulation gives (linear.ACCUMULATE_IN_PLACE = False: the same sums, formed
    then added in the same order)."""
    small = dict(d_model=64, num_queries=6, feature_dim=64, enc_layers=2, dec_layers=2, ff_dim=128, dropout=0.0)
    video, vmask, dur = PKG.dvc_core.synthetic_clips(2, T=512, feature_dim=64, padded=True, device=dev)
    audio, amask, _ = PKG.dvc_core.synthetic_clips(2, T=16, feature_dim=64, padded=True, seed=9, device=dev)
    batch = (video, vmask, audio, amask, dur)

    def run(in_place):
        monkeypatch.setattr(PKG.models.modules.linear, "ACCUMULATE_IN_PLACE", in_place)
        # (activation gradients as autograd sums them in both runs: test_grad_sum_in_gemm)
        monkeypatch.setattr(PKG.models.modules.linear, "GRAD_SUM_IN_GEMM", False)
        torch.manual_seed(0)
        model = PKG.dvc_core.MultimodalDVCCore(num_classes=5, **small).to(dev)
        tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.multimodal_workload_loss, lr=1e-3, use_bf16=True,
                                            graph=False)
        PKG._trace.clear()
        loss = tr._forward_backward(batch)
        torch.cuda.synchronize()
        return loss, tr.flat_grad.clone(), dict(PKG._trace.hits), [p.numel() for p in tr.params], tr._offs

    loss_r, ref, hits_r, sizes, offs = run(False)
    _, ref2, _, _, _ = run(False)
    loss, got, hits, _, _ = run(True)
    assert hits_r.get("grad_accum_view", 0) == 0 and hits_r.get("wgrad_into_grad", 0) == 0, hits_r
    assert hits.get("grad_accum_view", 0) > 0 and hits.get("wgrad_into_grad", 0) > 0, hits

    assert torch.equal(loss, loss_r)
    # not bit for bit: the decoders' per-tap MSDA backward sums each value row's list in the order its
    # atomics placed the taps, which varies run to run, and bf16 GEMMs carry that upstream (a
    # gradient cast to bf16 may round either way: the duration embedding's, a sum over every token).
    # So the in-place run must be as close to autograd's as two autograd runs are to each other, up
    # to 5e-3 of the gradient's norm (such flips reach the BaseEncoder's first convolution at ~1e-3
    # even when two runs happen to agree there) — far below a missing or doubled contribution of a
    # shared call (the audio stream's share of a shared weight's gradient is several percent).
    for i, (n, off) in enumerate(zip(sizes, offs)):
        a, b, c = got[off:off + n].double(), ref[off:off + n].double(), ref2[off:off + n].double()
        spread = (b - c).norm().item()
        assert (a - b).norm().item() <= 4 * spread + 5e-3 * b.norm().item() + 1e-9, i
