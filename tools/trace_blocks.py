#!/usr/bin/env python3
"""Group a rocprofv3 kernel trace into runs of consecutive launches of one MSDA kernel (the
microbenchmark calls each shape back to back) and print each run's median duration.
usage: trace_blocks.py run_kernel_trace.csv [name-regex]"""
import csv
import re
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"msda_bwd")
blocks = []
for r in rows:
    name = r["Kernel_Name"]
    if not pat.search(name):
        continue
    m = re.search(r"(msda_\w+?)<(.*?)>\(", name)
    short = f"{m.group(1)}<{m.group(2).replace('(anonymous namespace)::', '')}>" if m else name[:60]
    grid = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if blocks and blocks[-1][0] == (short, grid):
        blocks[-1][1].append(us)
    else:
        blocks.append(((short, grid), [us]))
for (short, grid), ts in blocks:
    print(f"{short[:58]:58s} wg={grid:6d} n={len(ts):3d} median_us={statistics.median(ts):8.2f} min_us={min(ts):8.2f}")
