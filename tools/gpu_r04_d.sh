#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/win_exp.py --regimes init,trained --exps 0,1,4,5 > gpurun_out/r04d_winexp.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_op.py -k "row_block or level_major or bench_instantiation or forward_tiles" > gpurun_out/r04d_win_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/determinism_diag.py > gpurun_out/r04c_det.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_prologue.py tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py tests/test_gpu_glue.py > gpurun_out/r04c_tests.log 2>&1
