"""The package Linear (models/modules/linear.py): same forward as nn.Linear, split-K fp32
weight gradient under bf16 autocast.  GPU cases compare with an fp64 reference computed from
the same bf16-rounded operands (the only rounding left is the bf16 forward output and the
fp32 accumulation order), and with stock autograd's bf16 gradient."""
import pytest
import torch

from conftest import PKG

linear_mod = PKG.models.modules.linear


def test_split_k_chunks():
    f = linear_mod.split_k_chunks
    assert f(15360) == 8
    assert f(8192) == 8
    assert f(4096) == 4
    assert f(2048) == 2
    assert f(800) == 1
    assert f(15361) == 1
    assert f(0) == 1


def test_cpu_is_plain_linear():
    torch.manual_seed(0)
    lin = linear_mod.Linear(16, 8)
    ref = torch.nn.Linear(16, 8)
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(3, 5, 16)
    torch.testing.assert_close(lin(x), ref(x), rtol=0, atol=0)
    assert set(lin.state_dict()) == {"weight", "bias"}


@pytest.mark.gpu
@pytest.mark.parametrize("tokens,n_in,n_out", [(15360, 512, 512), (15360, 512, 128), (800, 512, 2048),
                                               (7, 64, 30)])
def test_autocast_grads_match_fp64(dev, tokens, n_in, n_out):
    torch.manual_seed(0)
    lin = linear_mod.Linear(n_in, n_out).to(dev)
    x = torch.randn(1, tokens, n_in, device=dev, requires_grad=True)
    gy = torch.randn(1, tokens, n_out, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = lin(x)
    assert y.dtype == torch.bfloat16
    y.backward(gy.to(torch.bfloat16))
    # fp64 reference on the bf16-rounded operands autocast feeds the GEMMs
    xb = x.detach().to(torch.bfloat16).double().reshape(-1, n_in)
    wb = lin.weight.detach().to(torch.bfloat16).double()
    gb = gy.to(torch.bfloat16).double().reshape(-1, n_out)
    y_ref = xb @ wb.t() + lin.bias.detach().to(torch.bfloat16).double()
    torch.testing.assert_close(y.double().reshape(-1, n_out), y_ref, rtol=1e-2, atol=1e-2)
    gw_ref = gb.t() @ xb
    gbias_ref = gb.sum(0)
    assert lin.weight.grad.dtype == torch.float32
    torch.testing.assert_close(lin.weight.grad.double(), gw_ref, rtol=1e-5, atol=1e-5 * gw_ref.abs().max().item())
    torch.testing.assert_close(lin.bias.grad.double(), gbias_ref, rtol=1e-5, atol=1e-5 * gbias_ref.abs().max().item())
    gx_ref = (gb @ wb).reshape(x.shape)
    torch.testing.assert_close(x.grad.double(), gx_ref, rtol=2e-2, atol=2e-2 * gx_ref.abs().max().item())


@pytest.mark.gpu
def test_accumulates_into_existing_grad(dev):
    """Shared heads (the DVC wrapper reuses one Linear per decoder level) accumulate."""
    torch.manual_seed(1)
    lin = linear_mod.Linear(64, 32).to(dev)
    x = torch.randn(4096, 64, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        (lin(x).float().sum() + lin(x * 2).float().sum()).backward()
    xb = x.to(torch.bfloat16).double()
    x2b = (x * 2).to(torch.bfloat16).double()
    ref = xb.sum(0) + x2b.sum(0)
    torch.testing.assert_close(lin.weight.grad.double(), ref.expand(32, 64), rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
def test_bf16_shadow_is_bitwise_the_cast_and_expires(dev):
    torch.manual_seed(2)
    lin = linear_mod.Linear(64, 48).to(dev)
    x = torch.randn(300, 64, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y_cast = lin(x)
    lin.set_bf16_shadow(lin.weight.detach().to(torch.bfloat16), lin.bias.detach().to(torch.bfloat16))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y_shadow = lin(x)
    torch.testing.assert_close(y_shadow, y_cast, rtol=0, atol=0)
    with torch.no_grad():  # an in-place change to the master weight retires the shadow
        lin.weight.mul_(2)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y_new = lin(x)
    torch.testing.assert_close(y_new.float(), (x @ (lin.weight.t())).float() + lin.bias, rtol=2e-2, atol=5e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("K,N,dtype", [(15360, 512, torch.bfloat16), (800, 128, torch.bfloat16),
                                       (15360, 2048, torch.float16), (37, 8, torch.bfloat16), (0, 64, torch.bfloat16),
                                       (4096, 1536, torch.bfloat16), (4097, 512, torch.bfloat16),
                                       (801, 3072, torch.float16)])
def test_bias_grad_column_sum(dev, K, N, dtype):
    """mfl_colsum (the Linear's bias gradient): fp32 column sums of a 16-bit (K, N) matrix vs fp64
    (K <= 4096: the one-pass kernel; longer K: partials + final)."""
    g = torch.randn(K, N, device=dev).to(dtype)
    out = linear_mod._bias_grad(g)
    ref = g.double().sum(0)
    assert out.dtype == torch.float32
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("tokens", [15360, 800, 7])
@pytest.mark.parametrize("shadow", [False, True])
def test_linear_pair_matches_two_linears(dev, tokens, shadow):
    """linear_pair (the MSDA query projections: one input cast, one fused backward) gives the
    two layers' outputs and the same gradients as calling them one after the other; with the
    trainer's bf16 shadow too.  The input gradient sums the two layers' contributions inside
    one GEMM instead of adding two bf16 products, so it agrees to bf16 rounding."""
    torch.manual_seed(1)
    a, b = linear_mod.Linear(512, 128).to(dev), linear_mod.Linear(512, 128).to(dev)
    a2, b2 = linear_mod.Linear(512, 128).to(dev), linear_mod.Linear(512, 128).to(dev)
    a2.load_state_dict(a.state_dict())
    b2.load_state_dict(b.state_dict())
    if shadow:
        for m in (a, b, a2, b2):
            m.set_bf16_shadow(m.weight.detach().to(torch.bfloat16), m.bias.detach().to(torch.bfloat16))
    x = torch.randn(2, tokens // 2 if tokens > 7 else tokens, 512, device=dev)
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ga, gb = torch.randn(*x.shape[:-1], 128, device=dev), torch.randn(*x.shape[:-1], 128, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ya, yb = linear_mod.linear_pair(x1, a, b)
        za, zb = a2(x2), b2(x2)
    torch.testing.assert_close(ya, za, rtol=0, atol=0)
    torch.testing.assert_close(yb, zb, rtol=0, atol=0)
    ((ya.float() * ga).sum() + (yb.float() * gb).sum()).backward()
    ((za.float() * ga).sum() + (zb.float() * gb).sum()).backward()
    for p, q in ((a.weight, a2.weight), (a.bias, a2.bias), (b.weight, b2.weight), (b.bias, b2.bias)):
        assert p.grad.dtype == torch.float32
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-5, atol=1e-5 * q.grad.abs().max().item())
    torch.testing.assert_close(x1.grad, x2.grad, rtol=2e-2, atol=2e-2 * x2.grad.abs().max().item())


class _ShortK(torch.nn.Module):
    """Short-K layers of every deferred kind: a Linear, a linear pair, the query self-attention's
    in-projection (q / k | v row blocks of one weight) and a Linear used twice."""

    def __init__(self, e=64):
        super().__init__()
        L = PKG.models.modules.linear.Linear
        self.a, self.b, self.c, self.d = L(e, e), L(e, e // 2), L(e, e // 2), L(e // 2, e)
        self.mha = torch.nn.MultiheadAttention(e, 4, dropout=0.0)

    def forward(self, x):
        h = torch.relu(self.a(x))
        p, q = PKG.models.modules.linear.linear_pair(h, self.b, self.c)
        pq = torch.cat([p, q], -1)
        mask = torch.ones(x.shape[:2], dtype=torch.bool, device=x.device)
        sa = PKG.models.modules.attention.mha_self_attention(self.mha, pq, h, mask)
        return sa + self.d(p) + self.d(q)


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_trainer_batched_weight_grads_match_per_layer(dev, graph, monkeypatch):
    """FlatGradTrainer's backward with the short-K weight gradients queued and batched
    (linear.py deferred_weight_grads) gives the per-layer GEMMs' gradients, eager and
    graph-captured (lr 0: the capture's warm-up step leaves the parameters as they are)."""
    def run(defer_rows):
        monkeypatch.setattr(PKG.models.modules.linear, "DEFER_MAX_ROWS", defer_rows)
        torch.manual_seed(0)
        model = _ShortK().to(dev)
        x = torch.randn(4, 24, 64, device=dev)
        w = torch.randn(4, 24, 64, device=dev)
        tr = PKG.train_step.FlatGradTrainer(model, lambda out: (out.float() * w).sum(), graph=graph, lr=0.0,
                                            weight_decay=0.0)
        PKG._trace.clear()
        if graph:
            tr.capture((x,), warmup=1)
            tr._g_fb.replay()
        else:
            tr._forward_backward((x,))
        torch.cuda.synchronize()
        return torch.cat([v.reshape(-1) for v in tr.grad_views]), dict(PKG._trace.hits), [p.numel() for p in tr.params]

    ref, hits_ref, sizes = run(0)
    got, hits, _ = run(4096)
    assert hits_ref.get("wgrad_batched", 0) == 0
    assert hits.get("wgrad_batched", 0) >= 7  # a, b, c, in_proj q/k and v, out_proj, d twice
    off = 0
    for i, n in enumerate(sizes):
        a, b = got[off:off + n].double(), ref[off:off + n].double()
        assert (a - b).norm() <= 1e-4 * b.norm() + 1e-6, (i, n)
        off += n


@pytest.mark.gpu
def test_dvc_core_step_with_batched_weight_grads(dev, monkeypatch):
    """The bench core's step with the decoder's weight gradients batched: the deferred products
    ran and every gradient is within the step's own run-to-run spread of the per-layer step's
    (bf16 rounding amplifies arrival-order reductions elsewhere in the step)."""
    def run(defer_rows):
        monkeypatch.setattr(PKG.models.modules.linear, "DEFER_MAX_ROWS", defer_rows)
        torch.manual_seed(0)
        model = PKG.dvc_core.DeformableDVCCore(d_model=256, num_queries=20, enc_layers=2, dec_layers=2,
                                               ff_dim=512, dropout=0.0).to(dev)
        batch = PKG.dvc_core.synthetic_clips(2, T=64, feature_dim=512, device=dev)
        gen = torch.Generator(device=dev).manual_seed(5)
        wts = {}

        def loss_fn(out):
            total = 0.0
            for k in ("hs", "memory", "all_segments", "all_counts", "all_logits"):
                o = out[k].float()
                if k not in wts:
                    wts[k] = torch.randn(o.shape, generator=gen, device=dev)
                total = total + (o * wts[k]).sum()
            return total

        tr = PKG.train_step.FlatGradTrainer(model, loss_fn, graph=False)
        PKG._trace.clear()
        tr._forward_backward(batch)
        torch.cuda.synchronize()
        return torch.cat([v.reshape(-1) for v in tr.grad_views]), dict(PKG._trace.hits), [p.numel() for p in tr.params]

    ref, _, sizes = run(0)
    ref2, _, _ = run(0)
    got, hits, _ = run(4096)
    assert hits.get("wgrad_batched", 0) >= 2 * 8  # 8 products per decoder layer
    assert torch.isfinite(got).all()
    off, bad = 0, []
    for i, n in enumerate(sizes):
        a, b, c = (t[off:off + n].double() for t in (got, ref, ref2))
        scale = b.norm().item() + 1e-12
        noise, err = (c - b).norm().item() / scale, (a - b).norm().item() / scale
        if err > 4 * noise + (1e-2 if n >= 64 else 0.1):
            bad.append((i, n, err, noise))
        off += n
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,bias", [(800, 512, 512, True), (800, 256, 512, True), (532, 512, 512, False),
                                        (37, 256, 128, True), (1, 32, 32, True), (1024, 96, 64, False),
                                        (760, 512, 512, True), (100, 512, 384, True)])
def test_small_gemm_matches_fp32_product(dev, M, N, K, bias):
    """The short-M HIP GEMM (include/gemm_small.h) against the fp32 product of the same bf16
    operands, rounded once to bf16 (what addmm's fp32-accumulating GEMM returns): at most one bf16
    ulp apart (summation order), and against torch.addmm itself."""
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    x = torch.randn(M, K, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(dev, torch.bfloat16)
    b = torch.randn(N, generator=g).to(dev, torch.bfloat16) if bias else None
    y = linear_mod.small_addmm(b, x, w)
    assert y is not None and y.dtype == torch.bfloat16 and y.shape == (M, N)
    ref = x.float() @ w.float().t() + (b.float() if bias else 0.0)
    ulp = ref.abs().clamp_min(1e-30) * 2 ** -7
    assert ((y.float() - ref).abs() <= ulp + 1e-6).all()
    lib = torch.addmm(b, x, w.t()) if bias else torch.mm(x, w.t())
    assert ((y.float() - lib.float()).abs() <= 2 * ulp + 1e-6).all()


@pytest.mark.gpu
def test_small_gemm_strided_rows_and_refusals(dev):
    """Row strides (a slice of a wider matrix, as the decoder's in_proj q/k rows of W) and the
    shapes it leaves to the library (N % 32 != 0, more than SMALL_GEMM_MAX_ROWS rows)."""
    x = torch.randn(200, 512, device=dev).to(torch.bfloat16)
    w = torch.randn(1536, 512, device=dev).to(torch.bfloat16) / 20
    y = linear_mod.small_addmm(None, x, w[512:1024])
    torch.testing.assert_close(y.float(), (x.float() @ w[512:1024].float().t()), rtol=2 ** -7, atol=1e-3)
    assert linear_mod.small_addmm(None, x, w[:100]) is None
    assert linear_mod.small_addmm(None, x, w[:1024]) is None  # N > 512: hipBLASLt is ahead there
    assert linear_mod.small_addmm(None, torch.zeros(2048, 512, device=dev, dtype=torch.bfloat16), w) is None


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(800, 512, 512), (800, 256, 512), (532, 512, 512), (37, 128, 256), (1, 32, 32),
                                   (800, 512, 256), (760, 512, 96), (100, 384, 512)])
def test_small_gemm_nn_matches_fp32_product(dev, M, N, K):
    """The short-M NN GEMM (dX = dY . W, W row-major (N, K); B staged in LDS and read transposed)
    against the fp32 product of the same bf16 operands: at most one bf16 ulp apart."""
    g = torch.Generator(device="cpu").manual_seed(M * 3 + K)
    dy = torch.randn(M, N, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / N ** 0.5).to(dev, torch.bfloat16)
    y = linear_mod.small_mm_nn(dy, w)
    assert y is not None and y.shape == (M, K)
    ref = dy.float() @ w.float()
    assert ((y.float() - ref).abs() <= ref.abs() * 2 ** -7 + 1e-6).all()
    # a column slice of a wider weight (the in_proj q / k rows) keeps its row stride
    w2 = (torch.randn(N, 2 * K, generator=g) / N ** 0.5).to(dev, torch.bfloat16)
    y2 = linear_mod.small_mm_nn(dy, w2[:, :K])
    assert y2 is not None
    ref2 = dy.float() @ w2[:, :K].float()
    assert ((y2.float() - ref2).abs() <= ref2.abs() * 2 ** -7 + 1e-6).all()


@pytest.mark.gpu
def test_slab_and_column_sums_accumulate(dev):
    """mfl_sum_slabs_ex / mfl_colsum_ex (include/flat_adamw.h): grouped slab sums, and both sums
    added into an existing gradient (sum formed first, then added) — the in-place accumulation of a
    shared layer's weight / bias products (linear._accum_target)."""
    L = PKG.models.modules.linear
    g = torch.Generator(device=dev).manual_seed(5)
    part = torch.randn(3, 4, 64, 32, device=dev, generator=g)
    out = torch.randn(3, 64, 32, device=dev, generator=g)
    want = out + part.sum(1)
    L._sum_slabs(part.view(12, 64, 32), out, accumulate=True, groups=3)
    torch.testing.assert_close(out, want, rtol=1e-6, atol=1e-6)
    fresh = L._sum_slabs(part.view(12, 64, 32)[:4])
    torch.testing.assert_close(fresh, part[0].sum(0), rtol=1e-6, atol=1e-6)
    for k in (300, 9000):  # one-pass and partials + final column sums
        g2 = torch.randn(k, 512, device=dev, generator=g).bfloat16()
        base = torch.randn(512, device=dev, generator=g)
        want = base + g2.float().sum(0)
        L._bias_grad(g2, base, accumulate=True)
        torch.testing.assert_close(base, want, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("s", [1, 2, 7, 8, 9, 16, 17])
def test_slab_sum_is_the_sequential_sum(dev, s):
    """sum_slabs_kernel loads up to 8 slabs at once but adds them in slab order: bitwise the
    sequential fp32 sum part[0] + part[1] + ... for any slab count (partial last group of 8)."""
    L = PKG.models.modules.linear
    g = torch.Generator(device=dev).manual_seed(s)
    part = torch.randn(s, 96, 40, device=dev, generator=g) * torch.logspace(-3, 3, 40, device=dev)
    want = part[0].clone()
    for k in range(1, s):
        want += part[k]
    torch.testing.assert_close(L._sum_slabs(part), want, rtol=0, atol=0)
