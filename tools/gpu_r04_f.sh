#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/win_exp.py --regimes init,trained --exps 0,1,4,5,13,37,45 > gpurun_out/r04f_winexp.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_op.py -k "row_block or level_major or bench_instantiation or forward_tiles" tests/test_sparse.py > gpurun_out/r04f_win_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_glue.py -k "linear_group or base_encoder" tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py > gpurun_out/r04f_tests2.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config dvc --steps 10 --warmup 3 > gpurun_out/r04f_bench_dvc.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config sparse --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r04f_bench_sparse.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04f_bench.log 2>&1 || exit $?
AMD_SERIALIZE_KERNEL=3 timeout -k 10 120 python -u tools/gemm_small_probe.py > gpurun_out/r04f_gemm_probe.log 2>&1
