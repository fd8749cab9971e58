#!/bin/bash
# rocprofv3 kernel times of the MSDA backward for each library variant build_tmp/lib_<name>.so
# (A/B builds with -D switches); per-shape medians via tools/trace_blocks.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS=${MICRO_ARGS:-"--iters 10 --dtypes bf16 --regimes init --shapes enc,dec,xmod --kernels bwd_all,bwd_value"}
for lib in build_tmp/lib_*.so; do
  n=$(basename $lib .so)
  MSDA_HIP_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/lab_$n -o run --output-format csv -- \
    python3 tools/msda_microbench.py $ARGS > gpurun_out/lab_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/lab_$n.log; exit 1; }
  f=$(find gpurun_out/lab_$n -name "*kernel_trace.csv" | head -1)
  echo "== $n"; python3 tools/trace_blocks.py "$f" "msda_bwd_pair"
done
