#!/usr/bin/env python3
"""Debug: the deterministic-mode pair backward on the clustered case of tests/test_gpu_op.py,
run with a checking build (MSDA_HIP_LIB=build_tmp/check.so, -DMSDA_PAIR_CHECK)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_op import rand_case, clustered_locations  # noqa: E402
from conftest import PKG  # noqa: E402
from oracle import msda_oracle as O  # noqa: E402

shapes = [256, 128, 64, 32]
value, _, aw, gout = rand_case(shapes, 2, 8, 64, 300, 4, torch.bfloat16, seed=31)
loc = clustered_locations(2, 300, 8, shapes, 4, seed=32)
args = [t.cuda() for t in (value, loc, aw, gout)]
starts = O.level_starts(shapes)
r1 = PKG.msda.msda_backward(args[0], shapes, starts, args[1], args[2], args[3])
torch.cuda.synchronize()
r2 = PKG.msda.msda_backward(args[0], shapes, starts, args[1], args[2], args[3])
torch.cuda.synchronize()
print("equal:", [bool(torch.equal(a, b)) for a, b in zip(r1, r2)])
