#!/bin/bash
# PMC passes over the segment-attention kernels (tools/seg_attn_microbench.py, one variant:
# SEG_MB_VARIANT, default 3 = skewed clips, all keys live, dropout 0.1 — the DVC step's shape).
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/pmcs; mkdir -p $OUT; export TMPDIR=/tmp
export SEG_MB_VARIANT=${SEG_MB_VARIANT:-3}
run() { local name=$1; shift; rm -rf $OUT/$name
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- \
    python3 tools/seg_attn_microbench.py > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU
run sq2 SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
python3 - $OUT <<'PY'
import csv, glob, os, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for path in glob.glob(os.path.join(sys.argv[1], "*", "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(float); keys = {}
    for r in csv.DictReader(open(path)):
        if "seg_attn" not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        keys[r["Dispatch_Id"]] = r["Kernel_Name"].split("::")[1].split("(")[0]
    for (disp, c), v in per.items():
        acc[keys[disp]][c].append(v)
for k, cs in sorted(acc.items()):
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
