#!/usr/bin/env python3
"""Per-GEMM efficiency of one bench step (bf16 autocast, B=8, T=1024, eager so every GEMM is
attributable; argv[2] "multimodal" for configs[2]): every aten mm / addmm / bmm / baddbmm / convolution call grouped by input shapes,
its device time and its TFLOP/s against the bf16 dense MFMA peak (2.5 PFLOP/s,
MI355X_MICROARCH.md).  Writes a CSV (argv[1]) and prints the table.  Diagnostic only."""
import csv
import importlib
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = importlib.import_module("multimodal-feature-learning_amd")
PEAK = 2500.0  # TFLOP/s, dense bf16


def flops(name, shapes):
    try:
        if name in ("aten::mm",):
            (m, k), (_, n) = shapes[0], shapes[1]
            return 2 * m * k * n
        if name == "aten::addmm":
            (m, k), (_, n) = shapes[1], shapes[2]
            return 2 * m * k * n
        if name == "aten::bmm":
            (b, m, k), (_, _, n) = shapes[0], shapes[1]
            return 2 * b * m * k * n
        if name == "aten::baddbmm":
            (b, m, k), (_, _, n) = shapes[1], shapes[2]
            return 2 * b * m * k * n
    except (ValueError, IndexError, TypeError):
        return None
    return None


def main(out_csv, config="video"):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    dc = PKG.dvc_core
    if config == "multimodal":  # configs[2]: bench.py --config multimodal's model and batch
        model = dc.MultimodalDVCCore(d_model=512, num_queries=100, dropout=0.1).to(dev)
        tr = PKG.train_step.FlatGradTrainer(model, dc.multimodal_workload_loss, graph=False)
        video, mask, dur = dc.synthetic_clips(8, T=1024, device=dev)
        audio, amask, _ = dc.synthetic_clips(8, T=50, seed=2000, device=dev)
        batch = (video, mask, audio, amask, dur)
    else:
        model = dc.DeformableDVCCore(d_model=512, num_queries=100, dropout=0.1).to(dev)
        tr = PKG.train_step.FlatGradTrainer(model, dc.workload_loss, graph=False)
        batch = dc.synthetic_clips(8, T=1024, device=dev)
    for _ in range(3):
        tr.eager_step(batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        tr.eager_step(batch)
        torch.cuda.synchronize()
    rows = []
    total_dev = 0.0
    for ev in prof.key_averages(group_by_input_shape=True):
        if ev.key not in ("aten::mm", "aten::addmm", "aten::bmm", "aten::baddbmm", "aten::convolution",
                          "aten::convolution_backward"):
            continue
        shapes = [tuple(s) for s in ev.input_shapes if isinstance(s, (list, tuple))]
        dev_us = getattr(ev, "device_time_total", None)
        if dev_us is None:
            dev_us = ev.cuda_time_total
        f = flops(ev.key, shapes)
        per_call = dev_us / max(ev.count, 1)
        tf = (f / (per_call * 1e-6) / 1e12) if f and per_call > 0 else None
        total_dev += dev_us
        rows.append({"op": ev.key, "shapes": str(shapes[:3]), "calls": ev.count, "us_per_call": round(per_call, 2),
                     "us_total": round(dev_us, 1), "gflop_per_call": round(f / 1e9, 3) if f else "",
                     "tflops": round(tf, 1) if tf else "", "frac_of_peak": round(tf / PEAK, 3) if tf else ""})
    rows.sort(key=lambda r: -r["us_total"])
    tot_f = sum((float(r["gflop_per_call"] or 0) * r["calls"]) for r in rows)
    print(f"GEMM/conv device time per step: {total_dev / 1e3:.2f} ms; GEMM GFLOP per step {tot_f:.0f}; "
          f"average {tot_f / (total_dev * 1e-6) / 1e3 if total_dev else 0:.0f} TFLOP/s")
    for r in rows:
        print(f"{r['op']:>28} {r['calls']:>4} x {r['us_per_call']:8.1f} us = {r['us_total']:8.1f} us "
              f"{r['gflop_per_call']:>8} GF {r['tflops']:>7} TF/s  {r['shapes']}")
    with open(out_csv, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(rows)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gemm_census.csv", sys.argv[2] if len(sys.argv) > 2 else "video")
