#!/bin/bash
# rocprofv3 kernel times of the segment-attention kernels for each library build_tmp/lib_<name>.so
# (tools/seg_attn_microbench.py, variants SEG_AB_VARIANTS, default "3 4": skewed clips, all keys
# live / key windows, dropout 0.1), alternating the libraries twice on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for lib in build_tmp/lib_*.so; do
  n=$(basename $lib .so)
  for v in ${SEG_AB_VARIANTS:-3 4}; do
    o=gpurun_out/sab_${n}_v${v}_r${rep}
    SEG_MB_VARIANT=$v MSDA_HIP_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $o -o run --output-format csv -- \
      python3 tools/seg_attn_microbench.py > $o.log 2>&1 || { echo "$n v$v failed"; tail -5 $o.log; exit 1; }
    python3 - $o "$n v$v r$rep" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted((r for r in csv.DictReader(open(f)) if "seg_attn" in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows[6:]:
    k = r["Kernel_Name"].split("::")[1].split("(")[0]
    by.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(sys.argv[2], {k: round(sum(v) / len(v), 1) for k, v in by.items()}, flush=True)
PY
  done
done
done
