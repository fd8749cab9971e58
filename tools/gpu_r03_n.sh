#!/bin/bash
# full GPU suite, headline bench, DVC profile
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03n_pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/r03n_pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -n "^E \|FAILED" gpurun_out/r03n_pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r03n_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r03n_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dvc3 -o run --output-format csv -- python3 bench.py --config dvc --steps 12 --warmup 1 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r03n_prof_dvc.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/r03n_prof_dvc.log | cut -c1-200
exit $rc
