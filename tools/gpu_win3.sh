#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_op.py -k "row_block" > gpurun_out/win3_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/win3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/win_ab.py > gpurun_out/win3_ab.log 2>&1
rc=$?; cat gpurun_out/win3_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/win3_prof -o run --output-format csv -- python3 tools/win_ab.py > /dev/null 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/dvc_census.py > gpurun_out/dvc_census.log 2>&1
rc=$?; head -n 80 gpurun_out/dvc_census.log; exit $rc
