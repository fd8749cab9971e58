#!/usr/bin/env python3
"""Segment cross-attention kernels in isolation at the DVC step's shape (n = 6 levels x 28
segments, B = 8 clips, K = 1920 keys, Lq = 19, 8 heads): forward + backward per variant, for
rocprofv3 --stats to split per kernel.  Variants: attention dropout on / off, the segment -> clip
index uniform or skewed as the DVC's crop-of-crop composition makes it, keys all live or windows."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import PKG  # noqa: E402

SA = PKG.models.modules.seg_attention


def make(n=168, B=8, K=1920, Lq=19, H=8, skew=False, windows=False, seed=0):
    g = torch.Generator().manual_seed(seed)
    d = 64 * H
    dev = torch.device("cuda")
    q = torch.randn(n, Lq, d, generator=g).to(dev, torch.bfloat16)
    pk = torch.randn(B, K, d, generator=g).to(dev, torch.bfloat16)
    pv = torch.randn(B, K, d, generator=g).to(dev, torch.bfloat16)
    bk = torch.randn(d, generator=g).to(dev, torch.bfloat16)
    bv = torch.randn(d, generator=g).to(dev, torch.bfloat16)
    if skew:  # levels 1..5 read clips 0..2 only (index composed through the first segments' clips)
        index = torch.cat([torch.arange(28) * B // 28, torch.randint(0, 3, (n - 28,), generator=g)])
    else:
        index = torch.randint(0, B, (n,), generator=g)
    if windows:
        live = torch.zeros(n, K, dtype=torch.bool)
        for s in range(n):
            a = int(torch.randint(0, K - 400, (1,), generator=g))
            live[s, a:a + 400] = True
    else:
        live = torch.ones(n, K, dtype=torch.bool)
    keep = live.clone()
    return q, pk, pv, bk, bv, index.to(dev), keep.to(dev), (~live).to(dev)


def run(name, p, sort=True, **kw):
    q, pk, pv, bk, bv, index, keep, masked = make(**kw)
    order = torch.argsort(index, stable=True).to(torch.int32) if sort else None
    leaves = [t.clone().requires_grad_(True) for t in (q, pk, pv, bk, bv)]
    seed = torch.tensor([12345], dtype=torch.int64, device=q.device) if p > 0 else None
    gout = torch.randn_like(q)
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(6):
        if i == 2:
            start.record()
        out = SA._SegmentAttention.apply(*leaves, index, keep, masked, 8, 0.125, p, seed, order)
        out.backward(gout)
    end.record()
    torch.cuda.synchronize()
    print(f"{name:34s} fwd+bwd {start.elapsed_time(end) / 4 * 1e3:8.1f} us", flush=True)


VARIANTS = [
    ("uniform, all live, p=0, unsorted", 0.0, dict(sort=False)),
    ("uniform, all live, p=0", 0.0, {}),
    ("uniform, all live, p=0.1", 0.1, {}),
    ("skewed, all live, p=0.1", 0.1, dict(skew=True)),
    ("skewed, windows, p=0.1", 0.1, dict(skew=True, windows=True)),
    ("uniform, windows, p=0", 0.0, dict(windows=True)),
]


def main():
    only = os.environ.get("SEG_MB_VARIANT")  # an index into VARIANTS (PMC passes: one variant)
    for i, (name, p, kw) in enumerate(VARIANTS):
        if only is None or int(only) == i:
            run(name, p, **kw)


if __name__ == "__main__":
    main()
