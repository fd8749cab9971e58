#!/usr/bin/env python3
"""Where the row-block backward's time goes: win_bwd_kernel at the bench's encoder call (B=8,
T=1024 pyramid, bf16) with parts skipped through MSDA_HIP_WIN_EXP (profiling only; results
wrong): 1 = no grad_value MFMA / C build, 2 = no coordinate-gradient stores, 4 = no dots and no
coordinate gradients, 8 = no grad_out loads, 32 = no coordinate loads (synthetic locations).  HIP-event averages over --iters launches, plus the forward for reference."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from msda_microbench import make, timeit, msda  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--regimes", default="init,trained")
    ap.add_argument("--exps", default="0,1,2,4,5,7,13,37,45")
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--lq", type=int, default=0, help="queries (0: S, the encoder call; 577: the sparse encoder)")
    ap.add_argument("--qorders", default="1,0", help="MSDA_HIP_QORDER values (tile order of the queries)")
    ap.add_argument("--fwd-lds", default="0", help="MSDA_HIP_FWD_LDS values to time")
    ap.add_argument("--fwd-stage", default="1,2,0", help="MSDA_HIP_FWD_STAGE values (per-wave staged forward) to time")
    ap.add_argument("--lm", default="1,0", help="MSDA_HIP_WIN_LM values (persistent level-major kernel) to time")
    ap.add_argument("--lm-modes", default="0", help="MSDA_HIP_WIN_LM_MODE values (0 queue, 1 static, 2 one block a WG)")
    args = ap.parse_args()
    os.environ["MSDA_HIP_PROFILING"] = "1"  # (MSDA_HIP_WIN_EXP is refused without it)
    dev = torch.device("cuda", 0)
    shapes = [args.T, args.T // 2, args.T // 4, args.T // 8]
    S, M, P, B = sum(shapes), 8, 4, 8
    Lq = args.lq or S
    starts = [sum(shapes[:i]) for i in range(4)]
    for regime in args.regimes.split(","):
        value, loc, aw, gout = make(regime, B, Lq, shapes, M, P, torch.bfloat16, dev)
        for qo in args.qorders.split(","):
            os.environ["MSDA_HIP_QORDER"] = qo
            tag = {"regime": regime, "T": args.T, "Lq": Lq, "qorder": int(qo)}
            for flag in args.fwd_lds.split(","):
                os.environ["MSDA_HIP_FWD_LDS"] = flag
                us = timeit(lambda: msda.msda_forward(value, shapes, starts, loc, aw, want_tiles=True), args.iters)
                print(json.dumps({**tag, "kernel": "fwd_tiles", "lds": int(flag), "us": round(us, 2)}), flush=True)
            os.environ["MSDA_HIP_FWD_LDS"] = "0"
            _, tiles = msda.msda_forward(value, shapes, starts, loc, aw, want_tiles=True)
            lm = msda.LEVEL_MAJOR
            loc_m, aw_m = loc.permute(0, 2, 3, 1, 4).contiguous(), aw.permute(0, 2, 3, 1, 4).contiguous()
            for flag in args.fwd_stage.split(","):
                os.environ["MSDA_HIP_FWD_STAGE"] = flag
                us = timeit(lambda: msda.msda_forward(value, shapes, starts, loc_m, aw_m, want_tiles=True, layout=lm),
                            args.iters)
                print(json.dumps({**tag, "kernel": "fwd_tiles_level_major", "stage": int(flag), "us": round(us, 2)}),
                      flush=True)
            os.environ.pop("MSDA_HIP_FWD_STAGE", None)
            _, tiles_m = msda.msda_forward(value, shapes, starts, loc_m, aw_m, want_tiles=True, layout=lm)
            for flag in args.lm.split(","):
                os.environ["MSDA_HIP_WIN_LM"] = flag
                for mode in (args.lm_modes.split(",") if flag == "1" else ["-"]):
                    os.environ["MSDA_HIP_WIN_LM_MODE"] = mode if mode != "-" else "0"
                    us = timeit(lambda: msda.msda_backward(value, shapes, starts, loc_m, aw_m, gout, tiles=tiles_m,
                                                           layout=lm), args.iters)
                    print(json.dumps({**tag, "kernel": "bwd_win_level_major", "lm": int(flag), "mode": mode,
                                      "us": round(us, 2)}), flush=True)
            os.environ.pop("MSDA_HIP_WIN_LM", None)
            os.environ.pop("MSDA_HIP_WIN_LM_MODE", None)
            for e in args.exps.split(","):
                os.environ["MSDA_HIP_WIN_EXP"] = e
                us = timeit(lambda: msda.msda_backward(value, shapes, starts, loc, aw, gout, tiles=tiles), args.iters)
                print(json.dumps({**tag, "kernel": "bwd_win", "exp": int(e), "us": round(us, 2)}), flush=True)
            os.environ.pop("MSDA_HIP_WIN_EXP", None)
        os.environ.pop("MSDA_HIP_WIN_EXP", None)


if __name__ == "__main__":
    main()
