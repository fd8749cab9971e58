#!/usr/bin/env python3
"""The short-M HIP GEMM (models/modules/linear.py small_addmm / small_mm_nn) against torch.addmm /
torch.mm (hipBLASLt) at the decoder / caption-decoder / audio shapes: device time per call from 50
calls captured in a HIP graph, interleaved, median of 5."""
import importlib
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = importlib.import_module("multimodal-feature-learning_amd")
L = PKG.models.modules.linear


def timed(fn, iters=50):
    """Device time per call: ``iters`` calls captured in one HIP graph and replayed (no host
    launch overhead in the measurement, as in the training step's graphs)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000


def main():
    dev = torch.device("cuda", 0)
    for M, N, K in [(800, 512, 512), (800, 256, 512), (800, 1024, 512), (800, 2048, 512), (800, 512, 2048),
                    (800, 512, 1024), (532, 512, 512), (532, 2048, 512), (532, 512, 2048), (760, 512, 512),
                    (760, 2048, 512), (100, 512, 512), (1024, 512, 512)]:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        b = torch.randn(N, device=dev).to(torch.bfloat16)
        g = torch.randn(M, N, device=dev).to(torch.bfloat16)  # dgrad: g (M, N) . w (N, K)
        res = {"lib": [], "hip": [], "lib_dgrad": [], "hip_dgrad": []}
        for _ in range(5):
            res["lib"].append(timed(lambda: torch.addmm(b, x, w.t())))
            res["hip"].append(timed(lambda: L.small_addmm(b, x, w)))
            res["lib_dgrad"].append(timed(lambda: torch.mm(g, w)))
            res["hip_dgrad"].append(timed(lambda: L.small_mm_nn(g, w)))
        med = {k: round(statistics.median(v), 2) for k, v in res.items()}
        print(json.dumps({"M": M, "N": N, "K": K, "us": med, "hip_TFs": round(2 * M * N * K / med["hip"] / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
