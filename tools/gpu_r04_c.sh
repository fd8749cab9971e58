#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/determinism_diag.py > gpurun_out/r04c_det.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_prologue.py tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py tests/test_gpu_glue.py > gpurun_out/r04c_tests.log 2>&1
