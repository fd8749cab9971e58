#!/bin/bash
# round 4: determinism after the conv lowering; conv / level-major / DVC bf16 tests
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/determinism_diag.py > gpurun_out/r04b_det.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_glue.py -k base_encoder \
  tests/test_gpu_op.py -k "level_major or bench_instantiation or lds_staged" \
  tests/test_gpu_prologue.py tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py > gpurun_out/r04b_tests.log 2>&1
