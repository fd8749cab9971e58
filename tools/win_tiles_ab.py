#!/usr/bin/env python3
"""A/B of the row-block backward's dispatch order and of the forward-written tile intervals, at
the bench's encoder call (B=8, T=1024 pyramid, Lq=S=1920, bf16) and the configs[3] per-rank call
(T=4096), init and trained sampling (tools/msda_microbench.py).  Interleaved rounds in one process
(HIP events, 20 calls each): forward plain vs forward + tiles; backward with its own prepass under
the coarsest-first order (MSDA_HIP_WIN_ORDER=0) and the position-chunk order, and backward fed the
forward's tiles.  Prints the median of 5 rounds per variant."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from msda_microbench import PKG, make  # noqa: E402

msda = PKG.msda


def timed(fn, iters=20):
    for _ in range(3):
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
    os.environ["MSDA_HIP_BWD_WIN"] = "1"
    for shapes in ([1024, 512, 256, 128], [4096, 2048, 1024, 512]):
        S = sum(shapes)
        starts = [sum(shapes[:i]) for i in range(len(shapes))]
        for regime in ("init", "trained"):
            value, loc, aw, gout = make(regime, 8, S, shapes, 8, 4, torch.bfloat16, dev)
            _, tiles = msda.msda_forward(value, shapes, starts, loc, aw, want_tiles=True)
            variants = {
                "fwd": lambda: msda.msda_forward(value, shapes, starts, loc, aw),
                "fwd_tiles": lambda: msda.msda_forward(value, shapes, starts, loc, aw, want_tiles=True),
                "bwd_order0": ("0", lambda: msda.msda_backward(value, shapes, starts, loc, aw, gout)),
                "bwd_chunks": ("1", lambda: msda.msda_backward(value, shapes, starts, loc, aw, gout)),
                "bwd_chunks_tiles": ("1", lambda: msda.msda_backward(value, shapes, starts, loc, aw, gout,
                                                                      tiles=tiles)),
            }
            res = {k: [] for k in variants}
            for _ in range(5):
                for k, v in variants.items():
                    if isinstance(v, tuple):
                        os.environ["MSDA_HIP_WIN_ORDER"] = v[0]
                        v = v[1]
                    res[k].append(timed(v))
            os.environ["MSDA_HIP_WIN_ORDER"] = "1"
            nbytes = msda.algorithmic_bytes("bwd", 8, S, 8, 64, S, 4, 4, 2)
            med = {k: round(statistics.median(v), 2) for k, v in res.items()}
            med["frac_bwd_chunks_tiles"] = round(nbytes / (med["bwd_chunks_tiles"] * 1e-6) / 8e12, 4)
            print(json.dumps({"T": shapes[0], "regime": regime, "median_us": med}), flush=True)


if __name__ == "__main__" and not os.environ.get("WIN_SPLIT_AB"):
    main()


def split_ab():
    """Waves per row block (MSDA_HIP_WIN_SPLIT) on the calls with few row blocks: configs[2]'s video
    queries over the audio pyramid (T_a = 50: 8 blocks a (b, m)) — row-block path forced — against the
    pair kernel (MSDA_HIP_BWD_WIN=0) it takes by default."""
    dev = torch.device("cuda", 0)
    shapes, Lq = [50, 25, 13, 7], 1920
    S = sum(shapes)
    starts = [sum(shapes[:i]) for i in range(len(shapes))]
    for regime in ("init", "trained"):
        value, loc, aw, gout = make(regime, 8, Lq, shapes, 8, 4, torch.bfloat16, dev)
        f = lambda: msda.msda_backward(value, shapes, starts, loc, aw, gout)  # noqa: E731
        variants = [("pair", "0", "1"), ("win_w1", "1", "1"), ("win_w4", "1", "4"), ("win_w8", "1", "8")]
        res = {k: [] for k, _, _ in variants}
        outs = {}
        for _ in range(5):
            for k, win, split in variants:
                os.environ["MSDA_HIP_BWD_WIN"], os.environ["MSDA_HIP_WIN_SPLIT"] = win, split
                res[k].append(timed(f))
                outs[k] = f()
        os.environ.pop("MSDA_HIP_WIN_SPLIT")
        os.environ["MSDA_HIP_BWD_WIN"] = "1"
        err = {k: max(((a.float() - b.float()).norm() / b.float().norm()).item() for a, b in zip(outs[k], outs["pair"]))
               for k in outs}
        print(json.dumps({"call": "video->audio", "regime": regime,
                          "median_us": {k: round(statistics.median(v), 2) for k, v in res.items()},
                          "max_rel_diff_vs_pair": {k: round(v, 6) for k, v in err.items()}}), flush=True)


if __name__ == "__main__" and os.environ.get("WIN_SPLIT_AB"):
    split_ab()
