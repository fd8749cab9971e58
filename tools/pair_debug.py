#!/usr/bin/env python3
"""Debug helper: run one MSDA backward case through the HIP path and the oracle and print where
grad_attn / grad_loc / grad_value disagree (by level, clip, head, clamp status)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_op import rand_case, run_hip, _np  # noqa: E402
from oracle import msda_oracle as O  # noqa: E402

shapes, B, M, D, Lq, P = eval(sys.argv[1]) if len(sys.argv) > 1 else ([50, 25, 13, 7], 3, 8, 64, 95, 4)
padding = sys.argv[2] if len(sys.argv) > 2 else "border"
value, loc, aw, gout = rand_case(shapes, B, M, D, Lq, P, torch.float32, seed=102)
out, gv, gl, ga = run_hip(value, shapes, loc, aw, gout, padding)
r_gv, r_gl, r_ga = O.msda_backward(_np(value), shapes, _np(loc), _np(aw), _np(gout), padding=padding)
bad = ~np.isclose(_np(ga), r_ga, rtol=2e-5, atol=2e-5)
print("grad_attn bad", bad.sum(), "of", bad.size)
for name, ax in (("clip", 0), ("head", 2), ("level", 3), ("point", 4)):
    print(name, bad.sum(axis=tuple(i for i in range(5) if i != ax)))
Ts = np.array(shapes, dtype=np.float64).reshape(1, 1, 1, -1, 1)
y = np.clip(_np(loc) * Ts - 0.5, 0, Ts - 1)
print("clamped low bad", (bad & (y == 0)).sum(), "high", (bad & (y == Ts - 1)).sum(), "interior", (bad & (y > 0) & (y < Ts - 1)).sum())
print("query idx of bad (first 40):", np.nonzero(bad)[1][:40])
badv = ~np.isclose(_np(gv), r_gv, rtol=2e-4, atol=2e-4)
print("grad_value bad", badv.sum(), "of", badv.size)
if badv.any():
    bv = badv.any(axis=(2, 3))  # (B, S)
    starts = np.cumsum([0] + list(shapes))
    for l, T in enumerate(shapes):
        rows = np.nonzero(bv[0, starts[l]:starts[l + 1]])[0]
        print(f"level {l} T={T} bad rows clip0:", rows[:30], "count", len(rows))
    err = np.abs(_np(gv) - r_gv).max(axis=(2, 3))
    print("max err per row clip0 level0:", np.round(err[0, :shapes[0]], 3))
