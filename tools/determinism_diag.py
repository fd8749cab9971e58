#!/usr/bin/env python3
"""Find the first non-reproducible op of the bf16 DVC training step.

Runs the eager staged step (FlatGradTrainer._forward_backward on tests/test_gpu_dvc_step.py's small
model) twice on the same weights and inputs under a TorchDispatchMode that records, for every aten
op, a bitwise checksum of its tensor inputs and outputs.  The first op whose inputs are bitwise equal
across the two runs but whose outputs differ is a non-deterministic op; an op whose inputs differ
while every earlier recorded output matched was fed by a non-aten producer (a HIP kernel behind
ctypes) that differed.  Prints the first mismatches with the package source line that issued them.
"""
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode
from torch.utils._pytree import tree_flatten

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import PKG  # noqa: E402
from test_gpu_dvc_step import _small  # noqa: E402

_UNINIT = {"empty", "empty_like", "new_empty", "empty_strided", "new_empty_strided"}
_W = {}


def _weights(n, dev):
    w = _W.get(dev)
    if w is None or w.numel() < n:
        w = (torch.arange(max(n, 1 << 20), device=dev, dtype=torch.int64) % 65521) + 1
        _W[dev] = w
    return w[:n]


def checksum(t):
    if not isinstance(t, torch.Tensor) or t.is_sparse or t.is_complex() or t.device.type == "meta":
        return None
    x = t.detach()
    if x.numel() == 0:
        return torch.zeros((), dtype=torch.int64, device=x.device)
    x = x.contiguous().reshape(-1)
    b = x.to(torch.uint8) if x.dtype == torch.bool else x.view(torch.uint8)
    return (b.to(torch.int64) * _weights(b.numel(), b.device)).sum()


def where():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "multimodal-feature-learning_amd" in fr.filename or "/tools/" in fr.filename or "/tests/" in fr.filename:
            return f"{os.path.relpath(fr.filename, ROOT)}:{fr.lineno} {fr.name}"
    return "?"


class Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.log = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        ins = [checksum(t) for t in tree_flatten((args, kwargs))[0] if isinstance(t, torch.Tensor)]
        out = func(*args, **kwargs)
        name = func.overloadpacket.__name__
        outs = [] if name in _UNINIT else [checksum(t) for t in tree_flatten(out)[0] if isinstance(t, torch.Tensor)]
        shapes = [tuple(t.shape) for t in tree_flatten(out)[0] if isinstance(t, torch.Tensor)][:2]
        self.log.append((str(func), shapes, ins, outs, where()))
        return out


def _host(vals):
    return [None if v is None else int(v.item()) for v in vals]


def run_once(tr, obj, seed):
    torch.manual_seed(seed)
    rec = Rec()
    with rec:
        loss = tr._forward_backward((obj,))
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    log = [(f, s, _host(i), _host(o), w) for f, s, i, o, w in rec.log]
    return loss.item(), tr.flat_grad.clone(), log


def compare(a, b, limit=30):
    print(f"ops: run A {len(a)}, run B {len(b)}")
    shown = 0
    first_nondet = None
    for k, (ra, rb) in enumerate(zip(a, b)):
        if ra[0] != rb[0]:
            print(f"  [{k}] op sequence diverges: {ra[0]} vs {rb[0]} at {ra[4]} / {rb[4]}")
            break
        in_eq, out_eq = ra[2] == rb[2], ra[3] == rb[3]
        if in_eq and out_eq:
            continue
        tag = "NONDETERMINISTIC (same inputs)" if in_eq else "inputs differ"
        if not in_eq:
            tag += " " + str([i for i, (x, y) in enumerate(zip(ra[2], rb[2])) if x != y])
        if not out_eq:
            tag += "; outputs differ " + str([i for i, (x, y) in enumerate(zip(ra[3], rb[3])) if x != y])
        if in_eq and first_nondet is None:
            first_nondet = k
        if shown < limit:
            print(f"  [{k}] {ra[0]} {ra[1]} {tag} at {ra[4]}")
            shown += 1
    if first_nondet is not None:
        ra = a[first_nondet]
        print(f"first non-deterministic aten op: [{first_nondet}] {ra[0]} {ra[1]} at {ra[4]}")
    return first_nondet


def main():
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    model, obj = _small(dev)
    tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.StagedDVCLoss(obj, model), lr=1e-4, use_bf16=True,
                                        graph=False)
    tr._forward_backward((obj,))  # warm-up (plans, lazy state)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    la, ga, loga = run_once(tr, obj, 123)
    lb, gb, logb = run_once(tr, obj, 123)
    print(f"loss A {la!r} B {lb!r} equal={la == lb}")
    print(f"flat grad rel diff {((ga - gb).norm() / gb.norm()).item():.3g} bitwise={torch.equal(ga, gb)}")
    compare(loga, logb)


if __name__ == "__main__":
    main()
