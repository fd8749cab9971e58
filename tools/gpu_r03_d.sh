#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_linear.py tests/test_gpu_bf16_composition.py > gpurun_out/r03d_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/r03d_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err
rc=$?; head -c 200 gpurun_out/r03d_bench.json; echo; [ $rc -eq 0 ] || exit $rc
WIN_T=4096 bash tools/pmc_win.sh > gpurun_out/r03d_pmc4096.log 2>&1
rc=$?; tail -n 12 gpurun_out/r03d_pmc4096.log; [ $rc -eq 0 ] || exit $rc
WIN_T=1024 bash tools/pmc_win.sh > gpurun_out/r03d_pmc1024.log 2>&1
rc=$?; tail -n 3 gpurun_out/r03d_pmc1024.log; exit $rc
