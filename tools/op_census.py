#!/usr/bin/env python3
"""Census of the glue ops of one eager bench step (copies, casts, cats, reductions, fills, adds …):
each aten op with its argument shapes / dtypes and the innermost package frames that issued it
(backward ops of built-in autograd nodes carry no Python frame: their shapes name them), ranked
by output bytes.  A TorchDispatchMode sees every op of the forward and of the backward.

usage: op_census.py [--config video|dvc|sparse] [--top 80]"""
import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

GLUE = ("copy", "_to_copy", "cat", "sum", "add", "fill", "zero", "mul", "div", "sub", "clone", "contiguous",
        "stack", "index", "gather", "scatter", "where", "masked", "expand", "repeat", "mean", "neg", "exp",
        "pow", "sqrt", "cumsum", "ne", "eq", "lt", "gt", "le", "ge", "bitwise", "logical", "copy_", "full",
        "empty_strided", "new_zeros", "zeros", "ones", "arange", "select_backward", "slice_backward",
        "constant_pad", "nonzero", "sort", "argsort", "topk")


def sig(x):
    if isinstance(x, torch.Tensor):  # "~": not contiguous (a strided copy kernel)
        return f"{str(x.dtype).replace('torch.', '')}{list(x.shape)}{'' if x.is_contiguous() else '~'}"
    if isinstance(x, (list, tuple)):
        return "[" + ",".join(sig(y) for y in x[:4]) + ("…" if len(x) > 4 else "") + "]"
    return ""


def nbytes(out):
    if isinstance(out, torch.Tensor):
        return out.numel() * out.element_size()
    if isinstance(out, (list, tuple)):
        return sum(nbytes(o) for o in out)
    return 0


class Census(TorchDispatchMode):
    def __init__(self, pkg_dir, everything=False):
        super().__init__()
        self.pkg_dir = pkg_dir
        self.everything = everything
        self.rows = collections.defaultdict(lambda: [0, 0])

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func.overloadpacket.__name__)
        if self.everything or any(g in name for g in GLUE):
            fr = [f for f in traceback.extract_stack()[:-1] if self.pkg_dir in f.filename or "bench.py" in f.filename]
            where = " <- ".join(f"{os.path.relpath(f.filename, self.pkg_dir)}:{f.lineno}" for f in fr[::-1][:3])
            if not where:  # backward: the autograd node being run (accumulation adds run between nodes)
                node = torch._C._current_autograd_node()
                where = f"(node {node.name()})" if node is not None else "(autograd engine: input accumulation)"
            key = (name, " ".join(s for s in (sig(a) for a in args) if s), where)
            r = self.rows[key]
            r[0] += 1
            r[1] += nbytes(out)
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="video")
    ap.add_argument("--top", type=int, default=80)
    ap.add_argument("--cpu", action="store_true", help="fp32 on the host (the autograd structure: accumulation adds, "
                                                       "selects; not the GPU fast paths)")
    ap.add_argument("--extra", default="", help="more bench.py arguments, e.g. '--batch 1 --T 256'")
    ap.add_argument("--ops", default="", help="comma list: only these aten ops (e.g. sum,mean,norm)")
    ap.add_argument("--by", default="bytes", choices=["bytes", "count"], help="order of the listing")
    a = ap.parse_args()
    sys.argv = [sys.argv[0], "--config", a.config, "--graph", "0", "--cpu-baseline", "0"] + a.extra.split()
    import bench
    args = bench.parse()
    dev = torch.device("cpu") if a.cpu else torch.device("cuda", 0)
    model = bench.build_model(args, dev)
    batch = bench.build_batch(args, 0, dev)
    if a.cpu:
        from oracle.cpu_model import oracle_core
        ctx = oracle_core(bench.PKG)
        ctx.__enter__()
    else:
        bench.PKG._native.load_library()
    trainer = bench.PKG.train_step.FlatGradTrainer(model, bench.loss_fn(args, batch, model), lr=1e-4,
                                                   weight_decay=1e-4, max_norm=0.1, use_bf16=not a.cpu, graph=False)
    trainer.capture(batch)
    for _ in range(2):
        trainer.step(batch)
    if not a.cpu:
        torch.cuda.synchronize()
    c = Census(os.path.join(ROOT, "multimodal-feature-learning_amd"), everything=bool(a.ops))
    with c:
        trainer.step(batch)
    if not a.cpu:
        torch.cuda.synchronize()
    tot_n = sum(v[0] for v in c.rows.values())
    print(f"{a.config}: {tot_n} glue ops in one step, {sum(v[1] for v in c.rows.values()) / 1e6:.1f} MB written")
    keep = set(a.ops.split(",")) if a.ops else None
    items = [kv for kv in c.rows.items() if keep is None or kv[0][0] in keep]
    order = (lambda kv: -kv[1][1]) if a.by == "bytes" else (lambda kv: (-kv[1][0], -kv[1][1]))
    for (name, s, where), (n, b) in sorted(items, key=order)[:a.top]:
        print(f"{b / 1e6:8.2f} MB {n:4d}x  {name} {s[:110]}\n              {where}")


if __name__ == "__main__":
    main()
