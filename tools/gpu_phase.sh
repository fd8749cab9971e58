#!/bin/bash
# Pair-kernel phase timing (build_tmp/phase_lib.so, -DMSDA_PHASE_TIMING) and rocprof medians of
# build_tmp/lib_*.so at the encoder and Sparse-DETR encoder shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
MSDA_HIP_LIB=$PWD/build_tmp/phase_lib.so timeout -k 10 200 python3 -u tools/msda_microbench.py --iters 2 --dtypes bf16 \
  --regimes init --shapes ${PH_SHAPES:-enc,sparse} --kernels bwd_all > gpurun_out/phase.log 2>&1 || { echo "phase failed"; tail -5 gpurun_out/phase.log; exit 1; }
grep -E "^pair|^fused" gpurun_out/phase.log | sort | uniq | head -60
MICRO_ARGS="--iters 20 --dtypes bf16 --regimes init --shapes ${PH_SHAPES:-enc,sparse} --kernels bwd_all" bash tools/lib_ab.sh
