#!/usr/bin/env python3
"""Weight-gradient split-K layouts at the multimodal encoder's joint rows (K = 16,120 = 15,360 video +
760 audio tokens): fp32 dW = dY^T X as one strided-batched GEMM over s equal K chunks (+ one mm over
the r leftover rows), timed with HIP events over back-to-back repeats (the slab sum excluded: the
same for every layout).  Diagnostic for models/modules/linear.py::_weight_grad's chunking."""
import sys

import torch


def layout(g2, x2, s, c):
    k, n_out, n_in = x2.shape[0], g2.shape[1], x2.shape[1]
    r = k - s * c
    part = torch.empty((s + (1 if r else 0), n_out, n_in), dtype=torch.float32, device=g2.device)

    def run():
        torch.bmm(g2[:s * c].view(s, c, n_out).transpose(1, 2), x2[:s * c].view(s, c, n_in), out_dtype=torch.float32,
                  out=part[:s])
        if r:
            torch.mm(g2[s * c:].t(), x2[s * c:], out_dtype=torch.float32, out=part[s])
    return run


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    from conftest import PKG
    global L
    L = PKG.models.modules.linear
    PKG._native.load_library()
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 16120
    dev = torch.device("cuda", 0)
    exact = ((8, 2015), (10, 1612), (13, 1240), (20, 806), (26, 620), (31, 520), (40, 403))  # divisors of 16,120
    for n_out, n_in, cands in ((2048, 512, ((8, None), (8, 1984), (7, 2048), (8, 1920), (16, 1007), (16, 960)) + exact),
                               (512, 2048, ((8, None), (8, 1984), (7, 2048), (8, 1920), (16, 1007), (16, 960)) + exact),
                               (512, 512, ((16, None), (16, 1000), (16, 960), (15, 1024), (16, 1008), (32, 496),
                                           (32, 448), (8, 1984)) + exact),
                               (256, 512, ((16, None), (16, 1000), (16, 960), (15, 1024), (16, 1008), (32, 496)) + exact)):
        g2 = torch.randn(k, n_out, device=dev).to(torch.bfloat16)
        x2 = torch.randn(k, n_in, device=dev).to(torch.bfloat16)
        for s, c in cands:
            c = k // s if c is None else c
            if s * c > k:
                continue
            t = timeit(layout(g2, x2, s, c))
            part = torch.randn(s + (1 if k - s * c else 0), n_out * n_in, device=dev)
            ts = timeit(lambda: L._sum_slabs(part))
            print(f"dW {n_out}x{n_in} K={k}: s={s:2d} c={c:5d} r={k - s * c:5d}  {t:7.2f} us  "
                  f"+ slab sum {ts:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
