#!/usr/bin/env python3
"""Runs the row-block MFMA backward (MSDA_HIP_BWD_WIN=1) 3 times at the bench's encoder call
(B=8, T=1024 pyramid, Lq=S=1920, bf16, init sampling): the PMC passes of tools/pmc_win.sh."""
import os
import sys

import torch

os.environ["MSDA_HIP_BWD_WIN"] = os.environ.get("MSDA_HIP_BWD_WIN", "1")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from msda_microbench import PKG, make  # noqa: E402

T = int(os.environ.get("WIN_T", "1024"))
shapes = [T, T // 2, T // 4, T // 8]
S = sum(shapes)
starts = [0, T, T + T // 2, T + T // 2 + T // 4]
value, loc, aw, gout = make("init", 8, S, shapes, 8, 4, torch.bfloat16, torch.device("cuda", 0))
for _ in range(3):
    PKG.msda.msda_backward(value, shapes, starts, loc, aw, gout)
torch.cuda.synchronize()
print("ok")
