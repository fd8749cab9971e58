#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_op.py -k "row_block or T4096" > gpurun_out/r03c_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r03c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/win_ab.py > gpurun_out/r03c_ab.log 2>&1
rc=$?; cat gpurun_out/r03c_ab.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/op_census.py > gpurun_out/r03c_census.log 2>&1
rc=$?; echo "census rc=$rc"; exit $rc
