#!/usr/bin/env python3
"""Per-step kernel time of a graph-replayed training step from a rocprofv3 kernel trace: the
kernels between consecutive `flat_adamw_update` launches (one per step), averaged over the last
N steps, grouped by kernel name with launch counts and grid sizes.

usage: dvc_step_breakdown.py run_kernel_trace.csv [steps=3] [top=30]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ups = [i for i, r in enumerate(rows) if "flat_adamw_update" in r["Kernel_Name"]]
    if len(ups) < n + 1:
        raise SystemExit(f"only {len(ups)} steps in the trace")
    a, b = ups[-n - 1], ups[-1]
    seg = rows[a + 1:b + 1]
    wall = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / n / 1e6
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for r in seg:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"]][0] += d
        agg[r["Kernel_Name"]][1] += 1
        busy += d
    print(f"steps averaged: {n}; kernels/step {len(seg) / n:.0f}; busy {busy / n / 1e6:.2f} ms/step; "
          f"wall {wall:.2f} ms/step (update to update)")
    print(f"{'us/step':>9} {'calls':>6} {'us/call':>8}  kernel")
    for k, (d, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:top]:
        print(f"{d / n / 1e3:9.1f} {c / n:6.0f} {d / c / 1e3:8.2f}  {k[:140]}")


if __name__ == "__main__":
    main()
