#!/usr/bin/env python3
"""Weight-gradient GEMM probe (library defaults only, no TunableOp candidates): times
dW = dY^T X for the bench step's Linear shapes (K = B*S = 15360 tokens, bf16) through
  mm        torch.mm, hipBLASLt default heuristic (what autograd does today)
  mm_rb     torch.mm with the rocBLAS backend
  mm_f32    torch.mm(..., out_dtype=float32)
  bmm_sK    split-K: s strided-batched partial products then a sum (s in 4, 8, 16)
Prints one JSON line per (shape, variant): avg us and TFLOP/s."""
import json

import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dev = torch.device("cuda", 0)
    K = 15360
    for out_f, in_f in ((512, 512), (128, 512), (2048, 512), (512, 2048)):
        dy = torch.randn(K, out_f, device=dev, dtype=torch.bfloat16)
        x = torch.randn(K, in_f, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * K * out_f * in_f
        ref = torch.mm(dy.t().float(), x.float())
        variants = {
            "mm": lambda: torch.mm(dy.t(), x),
            "mm_f32": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32),
        }
        for s in (4, 8, 16):
            variants[f"bmm_s{s}"] = (lambda s=s: torch.bmm(dy.view(s, K // s, out_f).transpose(1, 2),
                                                           x.view(s, K // s, in_f)).float().sum(0))
        for name, fn in variants.items():
            us = timeit(fn)
            err = ((fn().float() - ref).abs().max() / ref.abs().max()).item()
            print(json.dumps({"out": out_f, "in": in_f, "K": K, "variant": name, "us": round(us, 2),
                              "TFLOPs": round(flops / us / 1e6, 1), "rel_err": round(err, 5)}), flush=True)
        torch.backends.cuda.preferred_blas_library("cublas")
        us = timeit(lambda: torch.mm(dy.t(), x))
        print(json.dumps({"out": out_f, "in": in_f, "K": K, "variant": "mm_rocblas", "us": round(us, 2),
                          "TFLOPs": round(flops / us / 1e6, 1)}), flush=True)
        torch.backends.cuda.preferred_blas_library("cublaslt")


if __name__ == "__main__":
    main()
