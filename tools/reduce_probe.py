#!/usr/bin/env python3
"""Times the small fp32 reductions autograd runs in the bench step (sum_to_size of broadcast
gradients), to find the ~30 us reduce_kernel launches of the step profile.  Diagnostic only."""
import torch

dev = torch.device("cuda", 0)


def t(fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


g1 = torch.randn(8, 100, 4, 1, device=dev)
g2 = torch.randn(8, 100, 512, device=dev)
g3 = torch.randn(6, 8, 100, 4, 1, device=dev)
print("sum_to_size (8,100,4,1)->(8,100,1,1): %.1f us" % t(lambda: g1.sum_to_size(8, 100, 1, 1)))
print("sum_to_size (8,100,4,1)->(8,1,4,1): %.1f us" % t(lambda: g1.sum_to_size(8, 1, 4, 1)))
print("sum over batch (8,100,512)->(100,512): %.1f us" % t(lambda: g2.sum(0)))
print("sum_to_size (8,100,512)->(1,100,512): %.1f us" % t(lambda: g2.sum_to_size(1, 100, 512)))
print("sum (8,100,512) all: %.1f us" % t(lambda: g2.sum()))
print("stacked (6,8,100,4,1)->(6,8,100,1,1): %.1f us" % t(lambda: g3.sum_to_size(6, 8, 100, 1, 1)))
