#!/bin/bash
# rocprof medians of the pair kernel for every build_tmp/lib_*.so (tools/lib_ab.sh) at AB_SHAPES.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
MICRO_ARGS="--iters 20 --dtypes bf16 --regimes init,trained --shapes ${AB_SHAPES:-enc,sparse} --kernels bwd_all" bash tools/lib_ab.sh
