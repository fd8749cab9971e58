#!/bin/bash
# GPU A/B session: op parity tests, then the MSDA microbenchmark on the default path and on the
# paths named in AB_PATHS (MSDA_HIP_BWD_PATH values).  Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest ${AB_TESTS:-tests/test_gpu_op.py} -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -5 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
ARGS=${MICRO_ARGS:-"--dtypes bf16,fp32 --regimes init,trained"}
timeout -k 10 200 python3 -u tools/msda_microbench.py $ARGS > gpurun_out/ab_default.log 2>&1 || exit $?
for p in ${AB_PATHS:-}; do
  timeout -k 10 200 env MSDA_HIP_BWD_PATH=$p python3 -u tools/msda_microbench.py $ARGS > gpurun_out/ab_$p.log 2>&1 || exit $?
done
grep -h '^{' gpurun_out/ab_*.log | head -100
