#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_glue.py -k "host_weights or linear_group or base_encoder" tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py > gpurun_out/r04g_tests2.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config dvc --steps 10 --warmup 3 > gpurun_out/r04g_bench_dvc.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config sparse --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r04g_bench_sparse.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r04g_bench.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config decode --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/r04g_bench_decode.log 2>&1 || exit $?
