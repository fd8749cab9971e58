#!/usr/bin/env python3
"""Decoder-sized GEMMs (800 query tokens = 8 clips x 100 queries) under hipBLASLt and rocBLAS
(torch.backends.cuda.preferred_blas_library), plus the encoder's 15360-token ones for reference:
HIP events over 50 calls each, bf16 in, the shapes and transposes the training step issues
(forward addmm, dgrad mm, wgrad mm with fp32 out)."""
import json

import torch


def t(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000


def main():
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    rows = []
    for M in (800, 15360):
        for (K, N) in ((512, 512), (512, 128), (512, 256), (512, 1024), (512, 2048), (2048, 512)):
            x = torch.randn(M, K, device=dev, dtype=bf)
            w = torch.randn(N, K, device=dev, dtype=bf)
            b = torch.randn(N, device=dev, dtype=bf)
            g = torch.randn(M, N, device=dev, dtype=bf)
            cases = {
                "fwd addmm": lambda: torch.addmm(b, x, w.t()),
                "dgrad mm": lambda: torch.mm(g, w),
                "wgrad mm fp32": lambda: torch.mm(g.t(), x, out_dtype=torch.float32),
            }
            for lib in ("cublaslt", "cublas"):
                torch.backends.cuda.preferred_blas_library(lib)
                for name, fn in cases.items():
                    try:
                        us = t(fn)
                    except Exception as e:  # noqa: BLE001
                        us = float("nan")
                        name += f" ({type(e).__name__})"
                    fl = 2 * M * K * N
                    rows.append(dict(M=M, K=K, N=N, lib="hipblaslt" if lib == "cublaslt" else "rocblas", op=name,
                                     us=round(us, 2), TFs=round(fl / (us * 1e-6) / 1e12, 1)))
                    print(json.dumps(rows[-1]), flush=True)
    torch.backends.cuda.preferred_blas_library("cublaslt")


if __name__ == "__main__":
    main()
