#!/usr/bin/env python3
"""Per-launch-shape summary of the MSDA kernels in a rocprofv3 --kernel-trace CSV.

rocprofv3 --stats aggregates every dispatch of a kernel symbol, which mixes the encoder
(Lq = S) and decoder (Lq = 100) calls of the same template instance.  This groups the
dispatches of each msda_* kernel by grid size (one grid size per call shape) and prints
count / avg / min / max duration plus VGPRs and LDS, so the bench's HIP-event
`avg_launch_ms` can be checked against the profiler per shape.

usage: tools/rocprof_msda_summary.py <run_kernel_trace.csv> [> profiles/<round>_msda_kernels.csv]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(msda_\w+?)<(.*?)>\(", name)
    if not m:
        return None
    args = m.group(2).replace("(anonymous namespace)::", "")
    return f"{m.group(1)}<{args}>"


def main(path):
    groups = defaultdict(list)
    meta = {}
    for r in csv.DictReader(open(path)):
        s = short(r["Kernel_Name"])
        if s is None:
            continue
        key = (s, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
        groups[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        meta[key] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"])
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid_x", "block_x", "calls", "avg_us", "min_us", "max_us", "vgpr", "agpr", "lds_bytes"])
    for key in sorted(groups, key=lambda k: -sum(groups[k])):
        d = groups[key]
        w.writerow([key[0], key[1], key[2], len(d), round(sum(d) / len(d) / 1e3, 2), round(min(d) / 1e3, 2),
                    round(max(d) / 1e3, 2), *meta[key]])


if __name__ == "__main__":
    main(sys.argv[1])
