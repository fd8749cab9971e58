#!/usr/bin/env python3
"""Weight-gradient probe for the bench step's Linear layers (library GEMMs only).

The training step keeps fp32 master weights whose gradients live in one flat fp32 buffer
(train_step.py); under bf16 autocast autograd computes dW = dY^T X in bf16, casts it to fp32
and adds it into p.grad (3 kernels, the GEMM without split-K).  Variants timed here, per
Linear shape (K = tokens of one step):
  autograd     mm (bf16 out) + cast + add_ into the fp32 grad     (today)
  addmm_f32    addmm(grad, dY^T, X, out_dtype=fp32, out=grad)      (one kernel, fp32 accumulate)
  splitK_s     baddbmm over s K-chunks with fp32 out, then sum into grad
  bias_sum     dY.sum(0) in bf16 + cast + add_                     (today)
  bias_mm      addmm(bias_grad, ones^T, dY, out_dtype=fp32)        (GEMV through the GEMM library)
Prints one JSON line per (shape, variant): avg us, TFLOP/s and the error vs an fp32 reference."""
import json
import sys

import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dev = torch.device("cuda", 0)
    shapes = [(15360, 512, 512), (15360, 128, 512), (15360, 2048, 512), (15360, 512, 2048),
              (800, 512, 512), (800, 2048, 512), (800, 512, 2048), (8192, 512, 512)]
    for K, out_f, in_f in shapes:
        g = torch.Generator(device="cpu").manual_seed(0)
        dy = torch.randn(K, out_f, generator=g).to(dev, torch.bfloat16)
        x = torch.randn(K, in_f, generator=g).to(dev, torch.bfloat16)
        grad = torch.zeros(out_f, in_f, device=dev)
        ref = torch.mm(dy.t().float(), x.float())
        flops = 2.0 * K * out_f * in_f

        def autograd_like():
            grad.add_(torch.mm(dy.t(), x).float())

        def addmm_f32():
            torch.addmm(grad, dy.t(), x, out_dtype=torch.float32, out=grad)

        variants = {"autograd": autograd_like, "addmm_f32": addmm_f32}
        for s in (2, 4, 8, 16):
            if K % s:
                continue
            part = torch.empty(s, out_f, in_f, device=dev)

            def split(s=s, part=part):
                torch.baddbmm(part, dy.view(s, K // s, out_f).transpose(1, 2), x.view(s, K // s, in_f),
                              beta=0, out_dtype=torch.float32, out=part)
                grad.add_(part.sum(0))
            variants[f"splitK_{s}"] = split
        for name, fn in variants.items():
            try:
                grad.zero_()
                fn()
                torch.cuda.synchronize()
                err = ((grad - ref).abs().max() / ref.abs().max()).item()
                us = timeit(fn)
            except Exception as e:  # report and continue
                print(json.dumps({"K": K, "out": out_f, "in": in_f, "variant": name, "error": str(e)[:200]}),
                      flush=True)
                continue
            print(json.dumps({"K": K, "out": out_f, "in": in_f, "variant": name, "us": round(us, 2),
                              "TFLOPs": round(flops / us / 1e6, 1), "rel_err": round(err, 6)}), flush=True)
        bgrad = torch.zeros(out_f, device=dev)
        ones = torch.ones(1, K, device=dev, dtype=torch.bfloat16)
        bref = dy.float().sum(0)
        bvars = {
            "bias_sum": lambda: bgrad.add_(dy.sum(0).float()),
            "bias_mm": lambda: torch.addmm(bgrad.view(1, -1), ones, dy, out_dtype=torch.float32,
                                           out=bgrad.view(1, -1)),
            "bias_sum_f32": lambda: bgrad.add_(dy.sum(0, dtype=torch.float32)),
        }
        for name, fn in bvars.items():
            try:
                bgrad.zero_()
                fn()
                torch.cuda.synchronize()
                err = ((bgrad - bref).abs().max() / bref.abs().max()).item()
                us = timeit(fn)
            except Exception as e:
                print(json.dumps({"K": K, "out": out_f, "variant": name, "error": str(e)[:200]}), flush=True)
                continue
            print(json.dumps({"K": K, "out": out_f, "variant": name, "us": round(us, 2), "rel_err": round(err, 6)}),
                  flush=True)
    sys.stdout.flush()


if __name__ == "__main__":
    main()
