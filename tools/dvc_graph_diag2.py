#!/usr/bin/env python3
"""bf16 run-to-run spread of the DVC step's gradient on fixed weights: eager vs eager, replay vs
replay, replay vs eager (relative norm of the flat-gradient difference), and the parameter groups
where replay and eager differ most."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_dvc_step import _small  # noqa: E402
from conftest import PKG  # noqa: E402


def main():
    for flag in os.environ.get("DIAG_SEG", "1,0").split(","):
        os.environ["MFL_SEG_ATTENTION"] = flag
        print(f"== MFL_SEG_ATTENTION={flag}")
        run()


def run():
    model, obj = _small(torch.device("cuda", 0))
    tg = PKG.train_step.FlatGradTrainer(model, PKG.dvc_core.StagedDVCLoss(obj, model), lr=1e-4, use_bf16=True,
                                        graph=True)
    tg.capture((obj,), warmup=1)

    def replay():
        tg._g_a.replay()
        torch.cuda.synchronize()
        tg.loss_fn.host(tg._stage_state, tg._request_host)
        tg.loss_fn.upload()
        tg._g_fb.replay()
        torch.cuda.synchronize()
        return tg._loss.item(), tg.flat_grad.clone()

    def eager():
        l = tg._forward_backward((obj,)).item()
        torch.cuda.synchronize()
        return l, tg.flat_grad.clone()

    r1, r2, e1, e2 = replay(), replay(), eager(), eager()
    rel = lambda a, b: ((a[1] - b[1]).norm() / b[1].norm()).item()  # noqa: E731
    print(f"losses replay {r1[0]:.6f} {r2[0]:.6f} eager {e1[0]:.6f} {e2[0]:.6f}")
    print(f"rel diff: replay-replay {rel(r1, r2):.4g} eager-eager {rel(e1, e2):.4g} replay-eager {rel(r1, e1):.4g}")
    names = {id(p): n for n, p in model.named_parameters()}
    groups = {}
    for i, p in enumerate(tg.params):
        k, off = p.numel(), tg._offs[i]
        g = ".".join(names[id(p)].split(".")[:3])
        a, b = r1[1][off:off + k], e1[1][off:off + k]
        d = groups.setdefault(g, [0.0, 0.0])
        d[0] += (a - b).norm().item() ** 2
        d[1] += b.norm().item() ** 2
    for g, (dd, bb) in sorted(groups.items(), key=lambda kv: -kv[1][0])[:12]:
        print(f"{g:40s} rel {(dd ** 0.5) / max(bb ** 0.5, 1e-12):.4g}  norm {bb ** 0.5:.4g}")


if __name__ == "__main__":
    main()
