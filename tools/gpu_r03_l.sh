#!/bin/bash
# segment cross-attention kernels: parity tests, then the DVC-related GPU tests and the DVC bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_seg_attention.py > gpurun_out/r03l_seg.log 2>&1
rc=$?; echo "seg rc=$rc"; tail -5 gpurun_out/r03l_seg.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dvc_step.py tests/test_dvc.py tests/test_add_norm.py -m gpu > gpurun_out/r03l_dvc.log 2>&1
rc=$?; echo "dvc rc=$rc"; tail -5 gpurun_out/r03l_dvc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config dvc --steps 20 --warmup 3 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r03l_bench_dvc.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/r03l_bench_dvc.log
exit $rc
