#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dvc_step.py tests/test_dvc.py -m gpu > gpurun_out/r03u_dvc.log 2>&1
rc=$?; echo "dvc rc=$rc"; tail -2 gpurun_out/r03u_dvc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config dvc --steps 20 --warmup 3 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r03u_bench_dvc.log 2>&1
rc=$?; echo "dvc bench rc=$rc"; tail -1 gpurun_out/r03u_bench_dvc.log | cut -c1-2000
exit $rc
