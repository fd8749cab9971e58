#!/bin/bash
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_glue.py -k base_encoder > gpurun_out/r04e_conv_test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/win_exp.py --regimes init,trained --exps 0,1,4,5,13,37,45 > gpurun_out/r04e_winexp.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_op.py -k "row_block or level_major or bench_instantiation or forward_tiles" > gpurun_out/r04e_win_tests.log 2>&1
