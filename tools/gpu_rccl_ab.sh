#!/bin/bash
# One GPU session: the train-step tests (RCCL one-rank capture smoke included), then the pair
# kernel A/B over build_tmp/lib_*.so at the encoder shape (tools/lib_ab.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_train_step.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train_step.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_train_step.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
MICRO_ARGS="--iters 20 --dtypes bf16 --regimes init,trained --shapes enc,xmod --kernels bwd_all" bash tools/lib_ab.sh
