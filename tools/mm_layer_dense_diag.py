#!/usr/bin/env python3
"""Diagnostic: the multimodal encoder layer of tests/test_add_norm.py::test_multimodal_layer_carry_matches_
uncarried run four ways — carried / uncarried bf16 operands x dense small-pyramid kernels on / off
(MSDA_HIP_DENSE) — printing, per parameter gradient, the relative difference of each run to the
carried + non-dense one, and a repeat of the dense run (determinism)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import PKG  # noqa: E402

MT = PKG.models.deformable.multimodal_deformable_transformer
AN = PKG.models.modules.add_norm


def main():
    dev = torch.device("cuda")
    torch.manual_seed(2)
    B, d, vs, as_ = 2, 512, [128, 64, 32, 16], [50, 25, 13, 7]
    layer = MT.MultimodalDeformableTransformerEncoderLayer(d, 1024, 0.0, "relu", 4, 8, 4).to(dev)

    def meta(shapes):
        ts = torch.tensor(shapes, device=dev)
        return ts, torch.cat([ts.new_zeros(1), ts.cumsum(0)[:-1]])
    vts, vlsi = meta(vs)
    ats, alsi = meta(as_)
    ones = torch.ones(B, 4, device=dev)
    vref = MT.MultimodalDeformableTransformerEncoder.get_reference_points(vts, ones, dev)
    aref = MT.MultimodalDeformableTransformerEncoder.get_reference_points(ats, ones, dev)
    v0, a0 = torch.randn(B, sum(vs), d, device=dev), torch.randn(B, sum(as_), d, device=dev)
    vp0, ap0 = torch.randn(B, sum(vs), d, device=dev), torch.randn(B, sum(as_), d, device=dev)
    wv, wa = torch.randn(d, device=dev), torch.randn(d, device=dev)
    carry_fn = MT.add_layer_norm_carry

    def uncarried(r, y, norm, pos=None, dropout=None):
        out = AN.add_layer_norm(r, y, norm, dropout)
        return out, out, None

    def run(carried, dense):
        os.environ["MSDA_HIP_DENSE"] = "1" if dense else "0"
        MT.add_layer_norm_carry = carry_fn if carried else uncarried
        layer.zero_grad(set_to_none=True)
        v, a = v0.clone().requires_grad_(True), a0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ov, oa = layer(v, vp0, vref, vts, vlsi, None, a, ap0, aref, ats, alsi, None)
        (ov.float() * wv).sum().add_((oa.float() * wa).sum()).backward()
        torch.cuda.synchronize()
        return [("v.grad", v.grad), ("a.grad", a.grad)] + [(n, p.grad.clone()) for n, p in layer.named_parameters()]

    runs = {name: run(c, dn) for name, (c, dn) in {
        "carried/nondense": (True, False), "uncarried/nondense": (False, False), "carried/dense": (True, True),
        "uncarried/dense": (False, True), "carried/dense again": (True, True)}.items()}
    base = runs["carried/nondense"]
    for name, other in runs.items():
        print(f"== {name} vs carried/nondense")
        for (n, a), (_, b) in zip(base, other):
            rel = ((a - b).norm() / a.norm().clamp_min(1e-30)).item()
            mx = ((a - b).abs().max() / a.abs().max().clamp_min(1e-30)).item()
            if rel > 1e-3 or mx > 4e-3:
                print(f"   {n:45s} rel {rel:.2e}  max/max {mx:.2e}")
    os.environ.pop("MSDA_HIP_DENSE", None)
    MT.add_layer_norm_carry = carry_fn
    # fp64 truth on the host (the oracle grid_sample core, oracle/cpu_model.py)
    import copy
    from oracle.cpu_model import oracle_core
    cpu = torch.device("cpu")
    lay64 = copy.deepcopy(layer).to(cpu).double()
    d64 = lambda t: t.detach().to(cpu).double()  # noqa: E731
    v, a = d64(v0).requires_grad_(True), d64(a0).requires_grad_(True)
    with oracle_core(PKG):
        ov, oa = lay64(v, d64(vp0), d64(vref), vts.cpu(), vlsi.cpu(), None, a, d64(ap0), d64(aref), ats.cpu(),
                       alsi.cpu(), None)
        (ov * d64(wv)).sum().add_((oa * d64(wa)).sum()).backward()
    truth = [("v.grad", v.grad), ("a.grad", a.grad)] + [(n, p.grad) for n, p in lay64.named_parameters()]
    print("== errors against the fp64 truth: |a - t| / |t| (norm), max |a - t| / max |t|")
    for name, other in runs.items():
        worst = []
        for (n, t), (_, g) in zip(truth, other):
            g = g.detach().to(cpu).double()
            rel = ((g - t).norm() / t.norm().clamp_min(1e-30)).item()
            mx = ((g - t).abs().max() / t.abs().max().clamp_min(1e-30)).item()
            worst.append((rel, mx, n))
        worst.sort(reverse=True)
        print(f"   {name:22s} " + "; ".join(f"{n} {r:.1e}/{m:.1e}" for r, m, n in worst[:4]))
        ab = dict((n, (g.detach().to(cpu).double(), t)) for (n, t), (_, g) in zip(truth, other))
        g, t = ab["self_attn.attention_weights.bias"]
        i = int((g - t).abs().argmax())
        print(f"      attention_weights.bias worst element {i}: got {g[i]:.4f} truth {t[i]:.4f} "
              f"(max |t| {t.abs().max():.2f})")


if __name__ == "__main__":
    main()
