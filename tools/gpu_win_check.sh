#!/bin/bash
# Row-block MFMA backward: parity against the oracle, then an A/B of the encoder-shape backward.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_op.py -k "row_block_mfma" > gpurun_out/win_tests.log 2>&1
rc=$?; tail -n 25 gpurun_out/win_tests.log; [ $rc -eq 0 ] || { echo "win tests rc=$rc"; exit $rc; }
timeout -k 10 300 python3 -u tools/win_ab.py > gpurun_out/win_ab.log 2>&1
rc=$?; cat gpurun_out/win_ab.log; exit $rc
