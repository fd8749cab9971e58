#!/usr/bin/env python3
"""Graph-replay check of the bench step with the HIP runtime's graph packet capture left ON
(DEBUG_CLR_GRAPH_PACKET_CAPTURE unset): five graph steps with allocating eager work (norms,
maxima) between the replays against five eager steps, as
tests/test_train_step.py::test_graph_steps_track_eager_steps_at_bench_shape, but bypassing the
trainer's capture guard.  Prints per step the graph / eager loss and gradient norm.  Run with the
variable unset in the environment: the package's setdefault must not turn the capture off, so
this script sets it to "1" before importing the package."""
import copy
import importlib
import os
import sys

os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = os.environ.get("PROBE_PACKET_CAPTURE", "1")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = importlib.import_module("multimodal-feature-learning_amd")
PKG.graph_packet_capture_off = lambda: True  # bypass the guard for this probe only

dev = torch.device("cuda", 0)
torch.manual_seed(0)
base = PKG.dvc_core.DeformableDVCCore(d_model=512, num_queries=100, dropout=0.0)
batch = PKG.dvc_core.synthetic_clips(8, T=1024, seed=1000, device=dev)
mk = lambda graph: PKG.train_step.FlatGradTrainer(copy.deepcopy(base).to(dev), PKG.dvc_core.workload_loss,  # noqa
                                                  lr=1e-4, weight_decay=1e-4, max_norm=0.1, use_bf16=True, graph=graph)
tg, te = mk(True), mk(False)
tg.capture(batch)
for _ in range(3):
    te.step(batch)
bad = 0
for i in range(5):
    lg = tg.step(batch).item()
    gg = tg.flat_grad.norm().item()
    le = te.step(batch).item()
    ge = te.flat_grad.norm().item()
    ok = abs(lg - le) <= 1e-2 * abs(le) + 1.0 and abs(gg - ge) <= 1e-2 * ge and gg == gg
    bad += not ok
    print(f"step {i}: graph loss {lg:.4f} gnorm {gg:.4f} | eager loss {le:.4f} gnorm {ge:.4f} {'ok' if ok else 'MISMATCH'}",
          flush=True)
print("packet capture", os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"], "mismatched steps:", bad)
