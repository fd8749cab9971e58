#!/usr/bin/env python3
"""Decoder value projections at the bench shape (memory 15360 x 512 bf16, six 512 x 512 layers):
six separate GEMMs vs one GEMM on the concatenated weights vs a batched GEMM whose A operand is
the same memory for every batch (stride 0), forward / dgrad / wgrad.  Diagnostic only."""
import torch

dev = torch.device("cuda", 0)
K, C, L = 15360, 512, 6
x = torch.randn(K, C, device=dev).bfloat16()
W = [torch.randn(C, C, device=dev).bfloat16() for _ in range(L)]
b = [torch.randn(C, device=dev).bfloat16() for _ in range(L)]
Wc = torch.cat(W, 0)
bc = torch.cat(b, 0)
G = torch.randn(L, K, C, device=dev).bfloat16()


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def sep_fwd():
    return [torch.addmm(b[i], x, W[i].t()) for i in range(L)]


def cat_fwd():
    return torch.addmm(bc, x, Wc.t())


Wt3 = torch.stack(W).transpose(1, 2)  # (L, C_in, C_out) view


def bmm_fwd():
    return torch.baddbmm(torch.stack(b)[:, None, :], x.expand(L, K, C), Wt3)


def bmm_fwd_nobias():
    return torch.bmm(x.expand(L, K, C), Wt3)


def sep_dgrad():
    acc = None
    for i in range(L):
        g = torch.mm(G[i], W[i]).float()
        acc = g if acc is None else acc + g
    return acc


def cat_dgrad():  # sum over layers inside one K = L*C GEMM
    return torch.mm(G.permute(1, 0, 2).reshape(K, L * C), Wc, out_dtype=torch.float32)


Gp = G.permute(1, 0, 2).contiguous().view(K, L * C)


def cat_dgrad_pre():
    return torch.mm(Gp, Wc, out_dtype=torch.float32)


def bmm_dgrad_sum():
    return torch.bmm(G, torch.stack(W), out_dtype=torch.float32).sum(0)


def sep_wgrad():
    out = []
    for i in range(L):
        part = torch.baddbmm(torch.empty(8, C, C, device=dev), G[i].view(8, K // 8, C).transpose(1, 2),
                             x.view(8, K // 8, C), beta=0, out_dtype=torch.float32)
        out.append(part.sum(0))
    return out


def bmm_wgrad():  # (L, C, K) x (K, C): dW_l = G_l^T x, one batched GEMM, split-K 2
    return torch.bmm(G.transpose(1, 2), x.expand(L, K, C), out_dtype=torch.float32)


def cat_wgrad():
    return torch.mm(Gp.t(), x, out_dtype=torch.float32)


flops_f = 2 * K * C * C * L
for name, fn in [("fwd 6 GEMMs", sep_fwd), ("fwd one GEMM (K x 3072)", cat_fwd), ("fwd bmm A stride 0", bmm_fwd),
                 ("fwd bmm no bias", bmm_fwd_nobias),
                 ("dgrad 6 GEMMs + fp32 adds", sep_dgrad), ("dgrad one GEMM K=3072 (permute)", cat_dgrad),
                 ("dgrad one GEMM pre-permuted", cat_dgrad_pre), ("dgrad bmm + sum", bmm_dgrad_sum),
                 ("wgrad 6 split-K", sep_wgrad), ("wgrad bmm", bmm_wgrad), ("wgrad one GEMM", cat_wgrad)]:
    try:
        us = timeit(fn)
        print(f"{name:>34}: {us:8.1f} us  {flops_f / us / 1e6:7.1f} TFLOP/s", flush=True)
    except Exception as ex:  # noqa: BLE001
        print(f"{name:>34}: failed {type(ex).__name__}: {ex}", flush=True)
y1 = torch.stack(sep_fwd())
y2 = bmm_fwd()
print("bmm fwd == separate:", torch.equal(y1, y2), "max diff", (y1.float() - y2.float()).abs().max().item())
print("expand stride kept:", x.expand(L, K, C).stride())
