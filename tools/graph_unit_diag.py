#!/usr/bin/env python3
"""Per-component HIP-graph replay check: captures fwd+bwd of one building block of the bench
step (MSDA core, fused prologue, autocast Linear, LayerNorm, Conv1d+GroupNorm, the whole
MSDeformAttn module), replays it, runs unrelated eager work (a reduction and a bf16 GEMM),
replays again and compares the gradients.  Diagnostic only."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = importlib.import_module("multimodal-feature-learning_amd")
dev = torch.device("cuda", 0)


def disturb():
    x = torch.randn(1024, 1024, device=dev)
    x.sum()
    torch.mm(x.bfloat16(), x.bfloat16())
    torch.cuda.synchronize()


def check(name, fn, leaves, same_stream=False, dump=None):
    """fn() -> scalar loss; leaves: tensors whose .grad is compared.  same_stream: warm up on
    the capture stream (else on a separate side stream)."""
    cs = torch.cuda.Stream()
    side = cs if same_stream else torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            for t in leaves:
                t.grad = None
            fn().backward()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    for t in leaves:
        t.grad = None
    g = torch.cuda.CUDAGraph()
    if dump:
        g.enable_debug_mode()
    with torch.cuda.graph(g, stream=cs):
        loss = fn()
        loss.backward()
    grads = [t.grad for t in leaves]
    if dump:
        g.debug_dump(dump)
        print("grad ptrs", [hex(x.data_ptr()) for x in grads], flush=True)
    g.replay()
    torch.cuda.synchronize()
    g1 = [x.clone() for x in grads]
    g.replay()
    torch.cuda.synchronize()
    g2 = [x.clone() for x in grads]
    disturb()
    g.replay()
    torch.cuda.synchronize()
    g3 = [x.clone() for x in grads]
    r12 = max(((a - b).norm() / (a.norm() + 1e-30)).item() for a, b in zip(g1, g2))
    r13 = max(((a - b).norm() / (a.norm() + 1e-30)).item() for a, b in zip(g1, g3))
    fin = all(bool(torch.isfinite(x).all()) for x in g3)
    print(f"{name:28s} replay-replay {r12:.3g}  after-eager {r13:.3g}  finite {fin}", flush=True)
    if not fin or r13 > 1e-2:
        for t in leaves:
            t.grad = None
        fn().backward()
        torch.cuda.synchronize()
        for i, t in enumerate(leaves):
            print(f"    leaf {i} {tuple(t.shape)} eager finite {bool(torch.isfinite(t.grad).all())} "
                  f"|eager|={t.grad.norm().item():.4g} g1 finite {bool(torch.isfinite(g1[i]).all())} "
                  f"|g1|={g1[i].norm().item():.4g} |g3|={g3[i].norm().item():.4g}", flush=True)


def main():
    torch.manual_seed(0)
    only = sys.argv[1] if len(sys.argv) > 1 else None
    if only == "mha2":
        import torch.nn.functional as F
        mha = torch.nn.MultiheadAttention(512, 8).to(dev)
        qm = torch.randn(100, 8, 512, device=dev, requires_grad=True)
        leaves = [qm] + [p for p in mha.parameters()]
        for nw in (True, False):
            def f(nw=nw):
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    return mha(qm, qm, qm, need_weights=nw)[0].float().square().mean()
            check(f"MHA need_weights={nw}", f, leaves)
        w, b = mha.in_proj_weight, mha.in_proj_bias

        def manual(stage, mode="autocast"):
            def f():
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode != "manual",
                                    cache_enabled=mode != "nocache"):
                    if mode == "manual":
                        proj = F.linear(qm.bfloat16(), w.bfloat16(), b.bfloat16())
                    elif mode == "fp32bias":
                        proj = F.linear(qm, w) + b
                    else:
                        proj = F.linear(qm, w, b)
                    proj = proj.unflatten(-1, (3, 512)).unsqueeze(0).transpose(0, -2).squeeze(-2).contiguous()
                    q, k, v = proj[0], proj[1], proj[2]
                    q = q.view(100, 64, 64).transpose(0, 1)
                    k = k.view(100, 64, 64).transpose(0, 1)
                    v = v.view(100, 64, 64).transpose(0, 1)
                    if stage == 0:
                        return (q.float().square().sum() + k.float().sum() + v.float().sum()) * 1e-3
                    a = torch.bmm(q * 0.125, k.transpose(-2, -1)).softmax(-1)
                    if stage == 1:
                        return a.float().square().mean()
                    o = torch.bmm(a, v).transpose(0, 1).contiguous().view(800, 512)
                    if stage == 2:
                        return o.float().square().mean()
                    o = F.linear(o, mha.out_proj.weight, mha.out_proj.bias)
                    return o.float().square().mean()
            return f
        for mode in ("manual", "nocache", "fp32bias"):
            check(f"stage 1 {mode}", manual(1, mode), [qm, w, b])
        for st_ in range(4):
            check(f"manual MHA stage {st_}", manual(st_), [qm, w, b] + ([mha.out_proj.weight, mha.out_proj.bias]
                                                                    if st_ == 3 else []))
        return
    if only == "mhadump":
        mha = torch.nn.MultiheadAttention(512, 8).to(dev)
        qm = torch.randn(100, 8, 512, device=dev, requires_grad=True)

        def mhaf():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return mha(qm, qm, qm)[0].float().square().mean()
        check("MHA dump", mhaf, [qm] + [p for p in mha.parameters()], dump="gpurun_out/mha_graph.dot")
        return
    if only == "lin3d":
        lin3d_cases()
        return
    if only == "reduce":
        reduce_cases()
        return
    if only == "mha":
        mha_cases()
        return
    B, S, M, D, Lq, L, P = 8, 1920, 8, 64, 1920, 4, 4
    shp, st = PKG.models.deformable.unimodal_deformable_transformer.level_metadata([1024, 512, 256, 128], dev)
    v = torch.randn(B, S, M, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    loc = torch.rand(B, Lq, M, L, P, device=dev, requires_grad=True)
    aw = torch.rand(B, Lq, M, L, P, device=dev, requires_grad=True)
    w = torch.randn(B, Lq, M * D, device=dev, dtype=torch.bfloat16)
    check("msda core", lambda: (PKG.msda.msda_apply(v, shp._mfl_host, st._mfl_host, loc, aw) * w).float().sum(), [v, loc, aw])

    off = torch.randn(B, Lq, M * L * P, device=dev, dtype=torch.bfloat16, requires_grad=True)
    logit = torch.randn(B, Lq, M * L * P, device=dev, dtype=torch.bfloat16, requires_grad=True)
    ref = torch.rand(B, Lq, L, 1, device=dev)
    wl = torch.randn(B, Lq, M, L, P, device=dev)

    def prol():
        lo, a = PKG.msda.msda_prologue_apply(off.view(B, Lq, M, L, P), logit.view(B, Lq, M, L * P), ref, shp._mfl_host)
        return (lo * wl).sum() + (a * wl).sum()
    check("prologue", prol, [off, logit])

    lin = PKG.models.modules.linear.Linear(512, 2048).to(dev)
    xin = torch.randn(B * S, 512, device=dev, requires_grad=True)

    def linf():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return lin(xin).float().square().mean()
    check("autocast Linear", linf, [xin, lin.weight, lin.bias])

    ln = torch.nn.LayerNorm(512).to(dev)
    xl = torch.randn(B, S, 512, device=dev, requires_grad=True)

    def lnf():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return ln(xl).float().square().mean()
    check("LayerNorm", lnf, [xl, ln.weight, ln.bias])

    conv = torch.nn.Sequential(torch.nn.Conv1d(512, 512, 3, 2, 1), torch.nn.GroupNorm(32, 512)).to(dev)
    xc = torch.randn(B, 512, 1024, device=dev, requires_grad=True)

    def convf():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return conv(xc).float().square().mean()
    check("Conv1d+GroupNorm", convf, [xc, conv[0].weight, conv[1].weight])

    attn = PKG.models.modules.attention.MSDeformAttn(512, L, M, P).to(dev)
    q = torch.randn(B, S, 512, device=dev, requires_grad=True)
    refp = torch.rand(B, S, L, 1, device=dev)

    def attf():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return attn(q, refp, q, shp, st, None).float().square().mean()
    check("MSDeformAttn", attf, [q] + [p for p in attn.parameters()])

    mha = torch.nn.MultiheadAttention(512, 8).to(dev)
    qm = torch.randn(100, B, 512, device=dev, requires_grad=True)

    def mhaf():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return mha(qm, qm, qm)[0].float().square().mean()
    check("MultiheadAttention", mhaf, [qm] + [p for p in mha.parameters()])


def lin3d_cases():
    import torch.nn.functional as F
    w = torch.randn(1536, 512, device=dev, requires_grad=True)
    b = torch.randn(1536, device=dev, requires_grad=True)
    x3 = torch.randn(100, 8, 512, device=dev, requires_grad=True)
    x2 = torch.randn(800, 512, device=dev, requires_grad=True)
    xt = torch.randn(8, 100, 512, device=dev).transpose(0, 1).detach().requires_grad_(True)

    def mk(x, post):
        def f():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = F.linear(x, w, b)
                if post:
                    y = y.unflatten(-1, (3, 512)).unsqueeze(0).transpose(0, -2).squeeze(-2).contiguous()
                    y = y[0] * y[1] + y[2]
                return y.float().square().mean()
        return f
    check("linear 2D", mk(x2, False), [x2, w, b])
    check("linear 3D", mk(x3, False), [x3, w, b])
    check("linear 3D non-contig", mk(xt, False), [xt, w, b])
    check("linear 3D + MHA split", mk(x3, True), [x3, w, b])

    def manual():
        y = F.linear(x3.bfloat16(), w.bfloat16(), b.bfloat16())
        return y.float().square().mean()
    check("linear 3D manual casts", manual, [x3, w, b])


def reduce_cases():
    """forward-only graphs of column / full reductions: replay, eager disturbance, replay"""
    cases = [((800, 1536), torch.bfloat16, (0,)), ((800, 1536), torch.float32, (0,)),
             ((100, 8, 1536), torch.bfloat16, (0, 1)), ((15360, 512), torch.bfloat16, (0,)),
             ((15360, 512), torch.float32, (0,)), ((8, 1024, 256), torch.float32, (1,)),
             ((1 << 20,), torch.float32, (0,)), ((4096, 4096), torch.float32, (0, 1))]
    for shape, dt, dims in cases:
        for out_f32 in (False, True):
            x = torch.randn(shape, device=dev).to(dt)
            kw = {"dtype": torch.float32} if out_f32 else {}
            x.sum(dims, **kw)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                y = x.sum(dims, **kw)
            g.replay()
            torch.cuda.synchronize()
            y1 = y.clone()
            ref = x.double().sum(dims)
            disturb()
            g.replay()
            torch.cuda.synchronize()
            err1 = ((y1.double() - ref).abs().max() / ref.abs().max()).item()
            err2 = ((y.double() - ref).abs().max() / ref.abs().max()).item()
            print(f"sum {shape} {dt} dims={dims} out_f32={out_f32}: replay err {err1:.3g}  after eager {err2:.3g}",
                  flush=True)


def mha_cases():
    B = 8
    for bias in (True, False):
        for ac in (True, False):
            mha = torch.nn.MultiheadAttention(512, 8, bias=bias).to(dev)
            qm = torch.randn(100, B, 512, device=dev, requires_grad=True)

            def mhaf():
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=ac):
                    return mha(qm, qm, qm)[0].float().square().mean()
            for same in (False, True):
                check(f"MHA bias={bias} autocast={ac} same={same}", mhaf, [qm] + [p for p in mha.parameters()],
                      same_stream=same)
    lin = torch.nn.Linear(512, 1536).to(dev)
    x = torch.randn(800, 512, device=dev, requires_grad=True)

    def linf():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return lin(x).float().square().mean()
    check("nn.Linear autocast", linf, [x, lin.weight, lin.bias])
    a = torch.randn(64, 100, 64, device=dev, requires_grad=True)

    def bmmf():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            s_ = torch.bmm(a, a.transpose(1, 2)).softmax(-1)
            return torch.bmm(s_, a).float().square().mean()
    check("bmm+softmax autocast", bmmf, [a])


if __name__ == "__main__":
    main()
