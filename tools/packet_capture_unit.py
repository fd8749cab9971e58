#!/usr/bin/env python3
"""Which captured node kind breaks under the HIP runtime's graph packet capture?

Each case captures a tiny graph around ONE node kind between two kernels, replays it, runs
allocating eager work (new tensors, a D2D clone, a reduction, a GEMM), replays again and checks
the result against the eager value.  Node kinds: a same-dtype D2D copy (hipMemcpyAsync, the
runtime's copyBuffer blit kernel), a hipMemsetAsync (the library's K=0 column-sum path), a
side-stream fork/join (event record / wait), a multi-block ATen sum, the library's K = 0 column
sum (a hipMemsetAsync until round 2, now a zero-fill kernel), and a plain kernel chain as the
control.
Run once with DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 and once with 0 (PROBE_PACKET_CAPTURE).
Diagnostic only."""
import importlib
import os
import sys

os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = os.environ.get("PROBE_PACKET_CAPTURE", "1")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = importlib.import_module("multimodal-feature-learning_amd")
dev = torch.device("cuda", 0)
N = 1 << 20


def disturb(k):
    a = torch.randn(N + 4096 * k, device=dev)
    b = a.clone()
    (a * b).sum()
    m = torch.randn(512, 512, device=dev).bfloat16()
    torch.mm(m, m)
    torch.cuda.synchronize()


def run_case(name, body, reps=4):
    x = torch.randn(N, device=dev)
    bufs = {"x": x, "tmp": torch.empty(N, device=dev), "out": torch.empty(N, device=dev),
            "col": torch.empty(256, device=dev)}
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            body(bufs)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    expect = bufs["out"].clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(bufs)
    bad = 0
    for k in range(reps):
        bufs["out"].fill_(-7.0)
        g.replay()
        torch.cuda.synchronize()
        err = (bufs["out"] - expect).abs().max().item()
        bad += not (err == 0.0)
        disturb(k)
    print(f"{name:>14}: {'OK' if bad == 0 else f'BAD in {bad}/{reps} replays'}", flush=True)
    return bad


def k_copy(b):
    b["tmp"].copy_(b["x"] * 2.0)          # kernel
    b["out"].copy_(b["tmp"])               # same dtype, contiguous: hipMemcpyAsync D2D
    b["out"].add_(1.0)                     # kernel


def k_chain(b):
    b["tmp"].copy_(b["x"] * 2.0)
    b["out"].copy_(b["tmp"] + 0.0)
    b["out"].add_(1.0)


_side = None


def k_fork(b):
    global _side
    if _side is None:
        _side = torch.cuda.Stream()
    cur = torch.cuda.current_stream()
    b["tmp"].copy_(b["x"] * 2.0)
    _side.wait_stream(cur)
    with torch.cuda.stream(_side):
        b["col"].copy_(b["tmp"][:256] * 3.0)
    cur.wait_stream(_side)
    b["out"].copy_(b["tmp"] + b["col"].sum())


def k_sum(b):  # a multi-block ATen reduction (its semaphores are zeroed with a memset)
    b["tmp"].copy_(b["x"] * 2.0)
    b["out"].copy_(b["tmp"] + b["tmp"].sum())


def k_colsum0(b):  # the library's K = 0 column sum, now a zero-fill kernel
    lib = PKG._native.load_library()
    b["tmp"].copy_(b["x"] * 2.0)
    assert lib.mfl_colsum(b["tmp"].data_ptr(), 0, 0, 256, b["col"].data_ptr(), b["tmp"].data_ptr(),
                          PKG._native.stream_handle(dev)) == 0
    b["out"].copy_(b["tmp"] + b["col"].sum())


def k_memset_raw(b):  # hipMemsetAsync itself, through the HIP runtime
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    b["tmp"].copy_(b["x"] * 2.0)
    b["col"].fill_(5.0)
    assert hip.hipMemsetAsync(ctypes.c_void_p(b["col"].data_ptr()), 0, ctypes.c_size_t(1024),
                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    b["out"].copy_(b["tmp"] + b["col"].sum())


bad = 0
for name, fn in (("kernel chain", k_chain), ("D2D memcpy", k_copy), ("hipMemsetAsync", k_memset_raw),
                 ("colsum K=0", k_colsum0), ("torch sum", k_sum), ("fork/join", k_fork)):
    bad += run_case(name, fn)
print("packet capture", os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"], "bad cases:", bad)
