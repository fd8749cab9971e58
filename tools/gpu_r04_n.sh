#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_seg_attention.py tests/test_dvc.py tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py tests/test_sparse.py > gpurun_out/r04n_tests.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04n_prof_seg -o run --output-format csv -- python3 tools/seg_attn_microbench.py > gpurun_out/r04n_seg_micro.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config dvc --steps 10 --warmup 3 --cpu-baseline 0 > gpurun_out/r04n_bench_dvc.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/op_census.py --config video --top 90 > gpurun_out/r04n_census_video.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/op_census.py --config dvc --top 140 > gpurun_out/r04n_census_dvc.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/op_census.py --config sparse --top 90 > gpurun_out/r04n_census_sparse.log 2>&1 || exit $?
MICRO_ARGS="--dtypes bf16 --regimes init --iters 3 --shapes enc --kernels fwd,bwd_all --layout level_major" timeout -k 10 900 bash tools/pmc_msda.sh > gpurun_out/r04n_pmc.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config sparse --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r04n_bench_sparse.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r04n_bench.log 2>&1
