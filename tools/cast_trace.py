#!/usr/bin/env python3
"""Where do the step's large copies / casts / adds come from?  One eager bench step (bf16
autocast, B=8, T=1024) under a dispatch mode that records every aten copy / cast / add / sum whose
output is at least 1 MB, with the innermost package frame that issued it (forward) or the
autograd node being run (backward).  Prints counts by (op, shape, dtype, origin).  Diagnostic only."""
import collections
import importlib
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = importlib.import_module("multimodal-feature-learning_amd")
WATCH = ("_to_copy", "copy_", "add", "add_", "sum", "clone", "cat", "masked_fill", "mul", "fill_", "zero_")


def origin():
    for fr in reversed(traceback.extract_stack()[:-3]):
        if "multimodal-feature-learning_amd" in fr.filename or "dvc_core" in fr.filename:
            return f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
    return "autograd engine"


class Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.__name__.split(".")[0]
        if name in WATCH and isinstance(out, torch.Tensor) and out.numel() * out.element_size() >= 1 << 20:
            src = [a.dtype for a in args if isinstance(a, torch.Tensor)]
            self.c[(name, tuple(out.shape), str(src[0]).replace("torch.", "") if src else "-",
                    str(out.dtype).replace("torch.", ""), origin())] += 1
        return out


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = PKG.dvc_core.DeformableDVCCore(d_model=512, num_queries=100, dropout=0.1).to(dev)
    tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.workload_loss, graph=False)
    batch = PKG.dvc_core.synthetic_clips(8, T=1024, device=dev)
    tr.eager_step(batch)
    rec = Rec()
    with rec:
        tr.eager_step(batch)
    torch.cuda.synchronize()
    tot = 0
    for (name, shape, a, b, org), n in sorted(rec.c.items(), key=lambda kv: -kv[1] * 1):
        print(f"{n:4d} {name:>12} {str(shape):>22} {a:>9}->{b:<9} {org}")
        tot += n
    print("total large ops:", tot)


if __name__ == "__main__":
    main()
