"""multimodal_bf16_d256: our stack's error against the reference fp64 run, per parameter, in bf16 (as the
GPU test runs it) and in fp32 (use_bf16=False: every kernel on its fp32 path) — whether a gradient's
bf16 error is noise of the 16-bit arithmetic or a systematic deviation (then fp32 shows it too).
usage: python tools/mm_fixture_diag.py [name-substring ...]"""
import importlib.util
import os
import sys

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import PKG  # noqa: E402

spec = importlib.util.spec_from_file_location("_mg", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
MG = importlib.util.module_from_spec(spec)
spec.loader.exec_module(MG)


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def run(use_bf16, g, dev):
    c = {k: int(v) for k, v in g["config"].items()}
    mods = MG.mm256_modules(PKG.models.deformable.multimodal_deformable_transformer.MultimodalDeformableTransformer,
                            PKG.models.modules.embedding_layers, PKG.models.base_encoder)
    MG.regen_parameters(mods, c["seed"])

    class S(nn.Module):
        def __init__(self, m):
            super().__init__()
            self.mods = m

        def forward(self, *a):
            return MG.mm256_forward(self.mods, *a)

    stack = S(mods).to(dev)
    video, vmask, audio, amask, durations, _ = MG.mm256_inputs()
    video, audio = video.to(dev).requires_grad_(True), audio.to(dev).requires_grad_(True)
    w = [t.to(dev) for t in g["weights"]]

    def loss_fn(out):
        return (out[2].float() * w[0]).sum() + (out[0].float() * w[1]).sum() + (out[1].float() * w[2]).sum()

    tr = PKG.train_step.FlatGradTrainer(stack, loss_fn, use_bf16=use_bf16, graph=False)
    tr._forward_backward((video, vmask.to(dev), audio, amask.to(dev), durations.to(dev)))
    torch.cuda.synchronize()
    res = {}
    for mname, grads in g["truth"]["grads"].items():
        params = dict(dict(mods.items())[mname].named_parameters())
        for k, t in grads.items():
            flat = params[k].grad.reshape(-1)
            s = flat[MG.grad_sample_index(mname + "." + k, flat.numel()).to(dev)]
            res[f"{mname}.{k}"] = (rel(s, t["sample"]), rel(g["bf16"]["grads"][mname][k]["sample"], t["sample"]))
    return res


def main():
    dev = torch.device("cuda", 0)
    g = torch.load(os.path.join(ROOT, "tests", "golden", "multimodal_bf16_d256.pt"), weights_only=True)
    keys = sys.argv[1:] or ["decoder.layers.0.cross_attn", "decoder.layers.1.cross_attn"]
    r16, r32 = run(True, g, dev), run(False, g, dev)
    for k in r16:
        if any(s in k for s in keys):
            print(f"{k:70s} bf16 {r16[k][0]:.5f}  fp32 {r32[k][0]:.2e}  reference bf16 {r16[k][1]:.5f}")
    print("max fp32 error over all sampled gradients: %.3e" % max(v[0] for v in r32.values()))


if __name__ == "__main__":
    main()
