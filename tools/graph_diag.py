#!/usr/bin/env python3
"""Graph-replay consistency check at the bench shape: replays the captured fwd+bwd graph
several times (with and without the update graph between) and compares each replay's
flat gradient with an eager fwd+bwd on the same parameters, per parameter.  Diagnostic only."""
import argparse
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = importlib.import_module("multimodal-feature-learning_amd")


def sizes(tr):
    return [p.numel() for p in tr.params]


def report(tag, tr, names, g, ref):
    rel = []
    for n, a, b in zip(names, g.split(sizes(tr)), ref.split(sizes(tr))):
        d = (a - b).norm().item()
        rel.append((d / (b.norm().item() + 1e-12), n, a.norm().item(), b.norm().item()))
    rel.sort(reverse=True)
    print(f"{tag}: |g|={g.norm().item():.6g} |ref|={ref.norm().item():.6g} worst:", flush=True)
    for r in rel[:6]:
        print(f"   rel={r[0]:.3g} {r[1]} |g|={r[2]:.4g} |ref|={r[3]:.4g}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dropout", type=float, default=0.0)
    ap.add_argument("--handover", type=int, default=1)
    ap.add_argument("--shadow", type=int, default=1)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = PKG.dvc_core.DeformableDVCCore(d_model=512, num_queries=100, dropout=args.dropout).to(dev)
    tr = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.workload_loss, lr=1e-4, weight_decay=1e-4, max_norm=0.1,
                                        use_bf16=True, graph=True, handover=bool(args.handover),
                                        shadow=bool(args.shadow))
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    assert len(names) == len(tr.params)
    batch = PKG.dvc_core.synthetic_clips(8, T=1024, seed=1000, device=dev)
    tr.capture(batch)

    def eager_fb():
        tr._forward_backward(batch)
        torch.cuda.synchronize()
        return tr.flat_grad.clone()

    def replay_fb():
        tr._g_fb.replay()
        torch.cuda.synchronize()
        return tr.flat_grad.clone()

    g1 = replay_fb()
    g2 = replay_fb()
    e0 = eager_fb()
    report("replay1 vs eager", tr, names, g1, e0)
    report("replay2 (no update) vs eager", tr, names, g2, e0)
    g3 = replay_fb()
    report("replay3 after eager fb vs eager", tr, names, g3, e0)
    tr._g_up.replay()
    torch.cuda.synchronize()
    g4 = replay_fb()
    e1 = eager_fb()
    report("replay after update vs eager", tr, names, g4, e1)
    tr._update()  # eager update, then graph fb
    torch.cuda.synchronize()
    g5 = replay_fb()
    e2 = eager_fb()
    report("replay after eager update vs eager", tr, names, g5, e2)


if __name__ == "__main__":
    main()
