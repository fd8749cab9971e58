#!/bin/bash
# deferred weight gradients + row-block default at T=4096: tests, then bench lines and a kernel census
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_linear.py tests/test_gpu_op.py tests/test_capi.py tests/test_gpu_bf16_composition.py > gpurun_out/r03b_tests.log 2>&1
rc=$?; tail -n 3 gpurun_out/r03b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err
rc=$?; head -c 420 gpurun_out/r03b_bench.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --T 4096 --steps 10 --warmup 3 > gpurun_out/r03b_bench_T4096.json 2> gpurun_out/r03b_bench_T4096.err
rc=$?; head -c 300 gpurun_out/r03b_bench_T4096.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03b_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > /dev/null 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
