#!/bin/bash
# rocprofv3 kernel times of the MSDA backward paths (default pair kernel vs AB_PATHS, e.g.
# "fused1 split") at the microbench call shapes; per-kernel / per-shape averages on stdout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS=${MICRO_ARGS:-"--iters 10 --dtypes bf16 --regimes init,trained --shapes enc,dec,enc4096,xmod --kernels bwd_all"}
for p in default ${AB_PATHS:-}; do
  env_p=""; [ "$p" != default ] && env_p="$p"
  MSDA_HIP_BWD_PATH=$env_p timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ab_$p -o run --output-format csv -- \
    python3 tools/msda_microbench.py $ARGS > gpurun_out/ab_$p.log 2>&1 || { echo "path $p failed"; tail -5 gpurun_out/ab_$p.log; exit 1; }
  f=$(find gpurun_out/ab_$p -name "*kernel_trace.csv" | head -1)
  echo "== $p"; python3 tools/rocprof_msda_summary.py "$f" | grep -E "^kernel|msda_bwd" | cut -d, -f1-7
done
