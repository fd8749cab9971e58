#!/usr/bin/env python3
"""Which parameters' gradients the trainer copies into the flat buffer after the backward (not
written in place by their producer: linear._claim), with their sizes — one eager step of a bench.py
workload.  Diagnostic for the per-bucket _foreach_copy_ of the step (profiles: multi_tensor_apply).

usage: claim_census.py [--config video|dvc|sparse]"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="video")
    a = ap.parse_args()
    sys.argv = [sys.argv[0], "--config", a.config, "--graph", "0", "--cpu-baseline", "0"]
    import bench
    args = bench.parse()
    dev = torch.device("cuda", 0)
    model = bench.build_model(args, dev)
    batch = bench.build_batch(args, 0, dev)
    bench.PKG._native.load_library()
    tr = bench.PKG.train_step.FlatGradTrainer(model, bench.loss_fn(args, batch, model), lr=1e-4, weight_decay=1e-4,
                                             max_norm=0.1, use_bf16=True, graph=False)
    names = {id(p): n for n, p in model.named_parameters()}
    copied = collections.Counter()
    orig = tr._flush_bucket

    def flush(b):
        _, _, idx = tr.buckets[b]
        for i in idx:
            p = tr.params[i]
            if p.grad is not None and p.grad.data_ptr() != tr.grad_views[i].data_ptr():
                copied[names.get(id(p), "?")] += p.numel()
        return orig(b)

    tr._flush_bucket = flush
    for _ in range(2):
        tr.eager_step(batch)
    copied.clear()
    tr.eager_step(batch)
    torch.cuda.synchronize()
    tot = sum(copied.values())
    print(f"{a.config}: {len(copied)} parameters copied after the backward, {tot / 1e6:.2f} M elements "
          f"({tot * 8 / 1e6:.1f} MB read + written)")
    kinds = collections.Counter()
    for n, c in copied.items():
        kinds[n.split(".")[-1] + " (" + ".".join(x for x in n.split(".")[:-1] if not x.isdigit())[-40:] + ")"] += c
    for k, c in kinds.most_common(40):
        print(f"  {c / 1e6:8.3f} M  {k}")


if __name__ == "__main__":
    main()
