#!/usr/bin/env python3
"""Where a graph-replayed staged DVC step (train_step.py, StagedDVCLoss) and the eager step differ:
on the same weights, one replay of graph A + host matching + graph B against one eager
_forward_backward (staged, and plain), bf16 autocast; per-parameter relative gradient differences,
largest first."""
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_dvc_step import _small  # noqa: E402
from conftest import PKG  # noqa: E402


def grads(tr):
    return {n: p.grad.detach().float().clone() if p.grad is not None else None
            for n, p in zip(tr._names, tr.params)}


def main():
    dev = torch.device("cuda", 0)
    bf16 = os.environ.get("DIAG_BF16", "1") == "1"
    model, obj = _small(dev)
    batch = (obj,)
    names = {id(p): n for n, p in model.named_parameters()}
    mg = copy.deepcopy(model)
    tg = PKG.train_step.FlatGradTrainer(mg, PKG.dvc_core.StagedDVCLoss(obj, mg), lr=1e-4, use_bf16=bf16, graph=True)
    tg._names = [dict((id(p), n) for n, p in mg.named_parameters())[id(p)] for p in tg.params]
    tg.capture(batch, warmup=1)
    # same weights: replay once, then an eager staged step on the same trainer
    tg._g_a.replay()
    torch.cuda.synchronize()
    tg.loss_fn.host(tg._stage_state, tg._request_host)
    tg.loss_fn.upload()
    tg._g_fb.replay()
    torch.cuda.synchronize()
    lg, fg = tg._loss.item(), tg.flat_grad.clone()
    le = tg._forward_backward(batch).item()
    fe = tg.flat_grad.clone()
    print(f"bf16={bf16} loss graph {lg:.6f} eager {le:.6f}; flat grad norm graph {fg.norm():.4f} eager {fe.norm():.4f}")
    off = 0
    rows = []
    for n, p in zip(tg._names, tg.params):
        k = p.numel()
        a, b = fg[off:off + k], fe[off:off + k]
        off += k
        rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
        rows.append((rel, n, a.norm().item(), b.norm().item()))
    rows.sort(reverse=True)
    for rel, n, na, nb in rows[:25]:
        print(f"{rel:9.4f}  graph {na:10.4f}  eager {nb:10.4f}  {n}")
    # plain (unstaged) eager on the same weights
    te = PKG.train_step.FlatGradTrainer(copy.deepcopy(mg), lambda r: PKG.dvc_core.dvc_workload_loss(r, obj),
                                        lr=1e-4, use_bf16=bf16, graph=False)
    lp = te._forward_backward(batch).item()
    print(f"plain eager loss {lp:.6f} grad norm {te.flat_grad.norm():.4f}")


if __name__ == "__main__":
    main()
