#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_op.py -k "position_order or bench_instantiation or row_block or level_major" tests/test_sparse.py > gpurun_out/r04i_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/win_exp.py --regimes init,trained --exps 0,1,4,5,13 > gpurun_out/r04i_winexp.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py > gpurun_out/r04i_tests2.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r04i_bench.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config sparse --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r04i_bench_sparse.log 2>&1
