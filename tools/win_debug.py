#!/usr/bin/env python3
"""Structured-input probes of the row-block MFMA backward (msda_win.hip) against the oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import importlib  # noqa: E402

PKG = importlib.import_module("multimodal-feature-learning_amd")
from oracle import msda_oracle as O  # noqa: E402

os.environ["MSDA_HIP_BWD_WIN"] = "1"
dev = torch.device("cuda", 0)


def run(value, shapes, loc, aw, gout):
    starts = O.level_starts(shapes)
    v, lc, a, g = (t.to(dev) for t in (value, loc, aw, gout))
    gv, gl, ga = PKG.msda.msda_backward(v, shapes, starts, lc, a, g)
    torch.cuda.synchronize()
    r = O.msda_backward(value.float().numpy(), shapes, loc.numpy(), aw.numpy(), gout.float().numpy())
    return [x.float().cpu().numpy() for x in (gv, gl, ga)], r


T, Lq = 64, 600
shapes = [T]
# queries q sample exactly at row q % 64 (y integer), aw = 1, P = 1
loc = ((torch.arange(Lq) % T).float() + 0.5) / T
loc = loc.view(1, Lq, 1, 1, 1).contiguous()
aw = torch.ones_like(loc)
value = torch.zeros(1, T, 1, 64).bfloat16()
for name, gout in (("gout=channel", torch.arange(64).float().view(1, 1, 64).expand(1, Lq, 64)),
                   ("gout=query%7", (torch.arange(Lq) % 7).float().view(1, Lq, 1).expand(1, Lq, 64))):
    (gv, gl, ga), (rgv, rgl, rga) = run(value, shapes, loc, aw, gout.contiguous().bfloat16())
    print(name, "max err", np.abs(gv - rgv).max())
    for row in (0, 1, 5, 17, 63):
        print("  row", row, "ours", gv[0, row, 0, :8], "ref", rgv[0, row, 0, :8])
# dots: value row r = r (all channels), gout = 1 -> d0 = 64 * base
value = torch.arange(T).float().view(1, T, 1, 1).expand(1, T, 1, 64).contiguous().bfloat16()
loc2 = ((torch.arange(Lq) % T).float() + 0.25) / T
loc2 = loc2.view(1, Lq, 1, 1, 1).contiguous()
gout = torch.ones(1, Lq, 64).bfloat16()
(gv, gl, ga), (rgv, rgl, rga) = run(value, shapes, loc2, aw, gout)
print("dots: ga max err", np.abs(ga - rga).max(), "gl max err", np.abs(gl - rgl).max())
print("  ga ours", ga.reshape(-1)[:8], "ref", rga.reshape(-1)[:8])
print("  gv max err", np.abs(gv - rgv).max())
