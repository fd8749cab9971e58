#!/bin/bash
# per-kernel times of the MSDA microbenchmark under rocprofv3 --kernel-trace --stats
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profmicro -o run --output-format csv -- \
  python3 tools/msda_microbench.py --iters 5 ${MICRO_ARGS:-} > gpurun_out/profmicro.log 2>&1
echo "rc=$?"
grep "{" gpurun_out/profmicro.log
