#!/usr/bin/env python3
"""Where does the full DVC training step (bench.py --config dvc) spend its time?  Eager steps under
torch.profiler: wall time vs summed device time, the aten ops by self CPU time and by device time,
and kernel launches per step.  Diagnostic only."""
import importlib
import os
import sys
import time

import torch
from torch.profiler import ProfilerActivity, profile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = importlib.import_module("multimodal-feature-learning_amd")


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = PKG.dvc_core.build_dvc(num_queries=100, T=1024, dropout=0.1).to(dev)
    batch = PKG.dvc_core.synthetic_dvc_batch(8, T=1024, seed=1000, device=dev)
    tr = PKG.train_step.FlatGradTrainer(model, lambda r: PKG.dvc_core.dvc_workload_loss(r, batch), graph=False)
    for _ in range(3):
        tr.eager_step((batch,))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        tr.eager_step((batch,))
    torch.cuda.synchronize()
    print(f"eager step wall: {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms")
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        tr.eager_step((batch,))
        torch.cuda.synchronize()
    ka = prof.key_averages()
    dev_total = sum(e.self_device_time_total for e in ka)
    n_kernels = sum(e.count for e in ka if e.device_type == torch.autograd.DeviceType.CUDA)
    print(f"device time (sum of kernels): {dev_total / 1e3:.2f} ms; kernels launched: {n_kernels}")
    print("--- by self CPU time")
    for e in sorted(ka, key=lambda e: -e.self_cpu_time_total)[:30]:
        print(f"{e.key[:70]:70s} calls={e.count:6d} self_cpu_ms={e.self_cpu_time_total / 1e3:8.3f}")
    print("--- by device time")
    for e in sorted(ka, key=lambda e: -e.device_time_total)[:30]:
        print(f"{e.key[:70]:70s} calls={e.count:6d} dev_ms={e.device_time_total / 1e3:8.3f}")


if __name__ == "__main__":
    main()
