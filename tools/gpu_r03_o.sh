#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_seg_attention.py > gpurun_out/r03q_seg.log 2>&1
rc=$?; echo "seg rc=$rc"; tail -3 gpurun_out/r03q_seg.log; [ $rc -eq 0 ] || { grep -n "^E " gpurun_out/r03q_seg.log | head; exit $rc; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dvc_step.py tests/test_dvc.py -m gpu > gpurun_out/r03q_dvc.log 2>&1
rc=$?; echo "dvc rc=$rc"; tail -2 gpurun_out/r03q_dvc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dvc6 -o run --output-format csv -- python3 bench.py --config dvc --steps 20 --warmup 3 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r03q_bench_dvc.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config dvc --steps 20 --warmup 3 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r03q_bench_dvc_plain.log 2>&1
rc=$?; echo "dvc bench rc=$rc"; tail -1 gpurun_out/r03q_bench_dvc_plain.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r03q_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r03q_bench.log | cut -c1-250
exit $rc
