#!/bin/bash
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_glue.py -k base_encoder > gpurun_out/r04e_conv_test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/win_exp.py --regimes init,trained --exps 0,1,4,5,13,37,45 > gpurun_out/r04e_winexp.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_op.py -k "row_block or level_major or bench_instantiation or forward_tiles" > gpurun_out/r04e_win_tests.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_glue.py -k linear_group tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py > gpurun_out/r04e_tests2.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config dvc --steps 10 --warmup 3 > gpurun_out/r04e_bench_dvc.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04e_bench.log 2>&1
