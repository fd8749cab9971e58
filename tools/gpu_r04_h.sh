#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py > gpurun_out/r04h_tests.log 2>&1 || exit $?
bash tools/pmc_win.sh > gpurun_out/r04h_pmc.log 2>&1
