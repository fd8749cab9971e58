#!/bin/bash
# round 4: row-block backward breakdown; level-major layout tests; DVC bf16 determinism
# diagnostic + the bf16 DVC step against the reference's bf16 run
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/win_exp.py > gpurun_out/r04a_winexp.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_op.py -k "level_major or bench_instantiation" tests/test_gpu_prologue.py > gpurun_out/r04a_lm_tests.log 2>&1
timeout -k 10 400 python -u tools/determinism_diag.py > gpurun_out/r04a_det.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py > gpurun_out/r04a_tests.log 2>&1
