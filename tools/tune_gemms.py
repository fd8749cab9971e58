#!/usr/bin/env python3
"""hipBLASLt / rocBLAS solution selection for the GEMM shapes of the bench step (PyTorch
TunableOp), in two phases so that nothing is tuned inside a training step:

  record: one eager bench step with TunableOp on and tuning OFF, recording every GEMM it issues
          (op, layout, sizes, leading dims) into an "untuned" CSV;
  tune:   the recorded plain and bias GEMMs (GemmTunableOp / GemmAndBiasTunableOp) are tuned
          offline with torch.cuda.tunable.tune_gemm_in_file; the winners go to --out
          (profiles/tunableop_gfx950.csv), which bench.py reads with tuning off.
Strided-batched GEMMs (GemmStridedBatchedTunableOp: split-K weight gradients, the decoder's
nn.MultiheadAttention bmm/baddbmm) are left to the default heuristics: tuning the attention
baddbmm inside a step hit a candidate solution that faulted (illegal address) on gfx950.
GPU only.

usage: tune_gemms.py record --untuned F | tune --untuned F --out OUT [--max-ms N]"""
import argparse
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KEEP = ("GemmTunableOp_", "GemmAndBiasTunableOp_")


def record(args):
    # the untuned file name is read when TunableOp initialises: set it before the first GEMM
    os.environ["PYTORCH_TUNABLEOP_UNTUNED_FILENAME"] = args.untuned
    pkg = importlib.import_module("multimodal-feature-learning_amd")
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(True)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = pkg.dvc_core.DeformableDVCCore(d_model=512, num_queries=100, dropout=0.1).to(dev)
    tr = pkg.train_step.FlatGradTrainer(model, pkg.dvc_core.workload_loss, graph=False)
    batch = pkg.dvc_core.synthetic_clips(args.batch, T=args.T, device=dev)
    tr.eager_step(batch)
    torch.cuda.synchronize()
    print("recorded GEMM calls of one step into", args.untuned, flush=True)


def tune(args):
    path = args.untuned
    if not os.path.exists(path):  # TunableOp inserts the device ordinal into the untuned file name
        path = path[:-4] + "0.csv" if path.endswith(".csv") else path + "0"
    lines = [ln for ln in open(path) if ln.strip()]
    kept = [ln for ln in lines if ln.startswith(KEEP)]
    uniq = sorted(set(kept))
    flt = args.untuned + ".plain.csv"
    with open(flt, "w") as fh:
        fh.writelines(uniq)
    print(f"{len(lines)} recorded GEMM calls, {len(uniq)} plain / bias GEMM shapes to tune "
          f"(strided-batched ones skipped)", flush=True)
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.record_untuned_enable(False)
    tun.set_max_tuning_duration(args.max_ms)
    tun.set_filename(args.out, insert_device_ordinal=False)
    torch.zeros(1, device="cuda")
    tun.tune_gemm_in_file(flt)
    print("tuned; results written to", args.out, "at exit", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("phase", choices=["record", "tune"])
    ap.add_argument("--untuned", default="gpurun_out/tunableop_untuned.csv")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "tunableop_gfx950.csv"))
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--max-ms", type=int, default=10, help="tuning time budget per GEMM (ms)")
    args = ap.parse_args()
    (record if args.phase == "record" else tune)(args)


if __name__ == "__main__":
    main()
