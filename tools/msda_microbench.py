#!/usr/bin/env python3
"""MSDA kernel microbenchmark: times each HIP kernel of the path through the C-ABI with
HIP events, at the bench's encoder / decoder call shapes (B=8, T=1024 pyramid, M=8, D=64,
L=4, P=4), for three location regimes:
  init     — the reference's initial sampling (ref point + integer offsets: every sample
             exactly on a map position),
  trained  — ref point + N(0, 2 / T_l) jitter (taps spread around the reference),
  uniform  — U(0, 1) locations (no locality at all).
Prints one JSON line per (dtype, shape, regime, kernel) with avg µs and algorithmic GB/s.
"""
import argparse
import importlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = importlib.import_module("multimodal-feature-learning_amd")
msda = PKG.msda


def make(regime, B, Lq, shapes, M, P, dtype, dev, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    S = sum(shapes)
    L = len(shapes)
    value = torch.randn(B, S, M, 64, generator=g).to(dev, dtype)
    if Lq == S:  # encoder: the reference points of every token (valid ratio 1)
        ref = torch.cat([(torch.arange(t, dtype=torch.float32) + 0.5) / t for t in shapes])
    elif Lq == 1920:  # cross-modal: the video tokens' reference points over the audio pyramid
        ref = torch.cat([(torch.arange(t, dtype=torch.float32) + 0.5) / t for t in (1024, 512, 256, 128)])
    else:  # the Sparse-DETR encoder's top-k tokens, handed over in position order
        ref = torch.rand(Lq, generator=g).sort()[0]
    ref = ref.view(1, Lq, 1, 1, 1).expand(B, Lq, M, L, P)
    T = torch.tensor(shapes, dtype=torch.float32).view(1, 1, 1, L, 1)
    theta = torch.arange(M, dtype=torch.float32) * (2 * 3.141592653589793 / M)
    d = torch.stack([theta.cos(), theta.sin()], -1)
    d = (d / d.abs().max(-1, keepdim=True)[0])[:, 0].view(1, 1, M, 1, 1)
    k = torch.arange(1, P + 1, dtype=torch.float32).view(1, 1, 1, 1, P)
    if regime == "init":
        loc = ref + d * k / T
    elif regime == "trained":
        loc = ref + d * k / T + torch.randn(B, Lq, M, L, P, generator=g) * 2.0 / T
    else:
        loc = torch.rand(B, Lq, M, L, P, generator=g)
    aw = torch.softmax(torch.randn(B, Lq, M, L * P, generator=g), -1).view(B, Lq, M, L, P)
    gout = torch.randn(B, Lq, M * 64, generator=g).to(dev, dtype)
    return value, loc.contiguous().to(dev), aw.to(dev), gout


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtypes", default="bf16,fp32")
    ap.add_argument("--regimes", default="init,trained,uniform")
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--shapes", default="enc,dec")
    ap.add_argument("--kernels", default="fwd,bwd_loc_aw,bwd_value,bwd_all,prologue_fwd,prologue_bwd")
    ap.add_argument("--layout", default="reference", choices=["reference", "level_major"],
                    help="coordinate layout of fwd / bwd_all (level_major: the bench step's encoder calls)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    M, L, P, D = 8, 4, 4, 64
    # (name, level shapes, Lq): configs[1] encoder / decoder calls, configs[3]'s T=4096 encoder
    # call, configs[2]'s video queries over the audio pyramid (T_a = 50)
    calls = [("enc", [1024, 512, 256, 128], 1920), ("dec", [1024, 512, 256, 128], 100),
             ("enc4096", [4096, 2048, 1024, 512], 7680), ("xmod", [50, 25, 13, 7], 1920),
             ("sparse", [1024, 512, 256, 128], 577)]
    for dname in args.dtypes.split(","):
        dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[dname]
        vb = 2 if dtype == torch.bfloat16 else 4
        for shape_name, shapes, Lq in calls:
            if shape_name not in args.shapes.split(","):
                continue
            S = sum(shapes)
            starts = [sum(shapes[:i]) for i in range(L)]
            for regime in args.regimes.split(","):
                value, loc, aw, gout = make(regime, args.B, Lq, shapes, M, P, dtype, dev)
                fwd_b = msda.algorithmic_bytes("fwd", args.B, S, M, D, Lq, L, P, vb)
                bwd_b = msda.algorithmic_bytes("bwd", args.B, S, M, D, Lq, L, P, vb)
                # as the training step runs them: the forward also writes the row-block backward's
                # tile intervals where that backward runs, and the backward reads them
                lay, lc, a = 0, loc, aw
                if args.layout == "level_major" and msda.level_major_ok(value, shapes, Lq, P):
                    lay = msda.LEVEL_MAJOR
                    lc, a = loc.permute(0, 2, 3, 1, 4).contiguous(), aw.permute(0, 2, 3, 1, 4).contiguous()
                _, tiles = msda.msda_forward(value, shapes, starts, lc, a, want_tiles=True, layout=lay)
                runs = {
                    "fwd": (lambda: msda.msda_forward(value, shapes, starts, lc, a, want_tiles=True, layout=lay),
                            fwd_b),
                    "bwd_loc_aw": (lambda: msda.msda_backward(value, shapes, starts, loc, aw, gout,
                                                              need_value=False), None),
                    "bwd_value": (lambda: msda.msda_backward(value, shapes, starts, loc, aw, gout,
                                                             need_loc=False, need_aw=False), None),
                    "bwd_all": (lambda: msda.msda_backward(value, shapes, starts, lc, a, gout, tiles=tiles, layout=lay),
                                bwd_b),
                }
                off = (torch.randn(args.B, Lq, M, L, P) * 2).to(dev, dtype)
                logits = torch.randn(args.B, Lq, M, L * P).to(dev, dtype)
                refp = torch.rand(args.B, Lq, L, 1, device=dev)
                ploc, paw = msda.prologue_forward(off, logits, refp, shapes)
                pro_b = args.B * Lq * M * L * P * (2 * vb + 2 * 4) + args.B * Lq * L * 4
                runs["prologue_fwd"] = (lambda: msda.prologue_forward(off, logits, refp, shapes), pro_b)
                runs["prologue_bwd"] = (lambda: msda.prologue_backward(loc, aw, paw, off, refp, shapes, True, True,
                                                                       True), pro_b + args.B * Lq * M * L * P * 4)
                for name, (fn, nbytes) in runs.items():
                    if name not in args.kernels.split(","):
                        continue
                    us = timeit(fn, args.iters)
                    rec = {"dtype": dname, "shape": shape_name, "regime": regime, "kernel": name,
                           "us": round(us, 2)}
                    if nbytes:
                        rec["alg_GBps"] = round(nbytes / (us * 1e-6) / 1e9, 1)
                    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
