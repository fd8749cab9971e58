#!/usr/bin/env python3
"""Per-step kernel time by category from a rocprofv3 --stats kernel_stats.csv of bench.py
(steps = calls of the encoder backward / 6).  usage: kstats.py run_kernel_stats.csv [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
steps = sum(int(r["Calls"]) for r in rows if "msda_bwd_pair_kernel" in r["Name"] or "win_bwd_kernel" in r["Name"] or "win_lm_kernel" in r["Name"]) / 6
cat = collections.Counter()
calls = collections.Counter()
for r in rows:
    n = r["Name"]
    t = float(r["TotalDurationNs"]) / 1e6 / steps
    if n.startswith("Cijk"):
        k = "gemm (hipBLASLt/Tensile)"
    elif "igemm" in n or "batched_transpose" in n:
        k = "conv (MIOpen)"
    elif "msda" in n or "win_" in n:
        k = "msda"
    elif "add_ln" in n:
        k = "add_ln"
    elif "spin_kernel" in n:
        k = "spin"
    elif "copy" in n.lower() or "Cat" in n or "convert" in n.lower():
        k = "copy/cast/cat"
    elif "elementwise" in n:
        k = "elementwise"
    elif "reduce" in n:
        k = "reduce"
    elif "colsum" in n or "sum_slabs" in n:
        k = "colsum"
    else:
        k = "other"
    cat[k] += t
    calls[k] += int(r["Calls"]) / steps
print(f"steps {steps:.1f}; total {sum(v for k, v in cat.items() if k != 'spin'):.3f} ms/step")
for k, v in cat.most_common():
    print(f"{v:7.3f} ms {calls[k]:6.0f} calls  {k}")
print("--- top kernels (ms/step, calls/step, avg us)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:7.3f} {int(r['Calls']) / steps:6.1f} {float(r['AverageNs']) / 1e3:8.1f}  {r['Name'][:100]}")
