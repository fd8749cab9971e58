#!/usr/bin/env python3
"""A/B of the bf16 encoder backward: pair-pull kernel (MSDA_HIP_BWD_WIN=0) against the row-block
MFMA kernel (=1), HIP events over 20 calls, at the bench's encoder call (B=8, T=1024 pyramid,
Lq=S=1920, M=8, D=64, P=4) and the configs[3] per-rank call (T=4096, S=Lq=7680), for the init and
trained sampling regimes of tools/msda_microbench.py.  Also checks the two paths agree."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from msda_microbench import PKG, make  # noqa: E402

msda = PKG.msda


def run(win, args, iters=20):
    os.environ["MSDA_HIP_BWD_WIN"] = win
    value, shapes, starts, loc, aw, gout = args
    f = lambda: msda.msda_backward(value, shapes, starts, loc, aw, gout)  # noqa: E731
    for _ in range(3):
        r = f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000, r


def main():
    dev = torch.device("cuda", 0)
    cases = [("enc", [1024, 512, 256, 128], 1920), ("enc", [4096, 2048, 1024, 512], 7680),
             ("video->audio", [50, 25, 13, 7], 1920)]  # configs[2]: video queries on the audio pyramid
    for name, shapes, Lq in cases:
        T = shapes[0]
        S = sum(shapes)
        starts = [sum(shapes[:i]) for i in range(len(shapes))]
        for regime in ("init", "trained"):
            value, loc, aw, gout = make(regime, 8, Lq, shapes, 8, 4, torch.bfloat16, dev)
            args = (value, shapes, starts, loc, aw, gout)
            t_pair, r_pair = run("0", args)
            t_win, r_win = run("1", args)
            err = [((a.float() - b.float()).norm() / b.float().norm()).item() for a, b in zip(r_win, r_pair)]
            nbytes = msda.algorithmic_bytes("bwd", 8, S, 8, 64, Lq, 4, 4, 2)
            print(json.dumps({"call": name, "T": T, "Lq": Lq, "regime": regime, "pair_us": round(t_pair, 2), "win_us": round(t_win, 2),
                              "win_frac": round(nbytes / (t_win * 1e-6) / 8e12, 4),
                              "rel_diff_gv_gl_ga": [round(e, 6) for e in err]}), flush=True)


if __name__ == "__main__":
    main()
