#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 4 | cut -c1-900; if [ $rc -ne 0 ]; then exit $rc; fi; }
run r03h_tests 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_op.py tests/test_gpu_prologue.py tests/test_gpu_bf16_composition.py tests/test_gpu_dvc_step.py tests/test_dvc.py \
  tests/test_train_step.py tests/test_gpu_linear.py \
  -m gpu -k "tiles or orders or row_block or T4096 or prologue or composition or dvc or staged or cross or train or graph or linear or wgrad or gemm"
run r03h_gemm_ab 200 python3 -u tools/small_gemm_ab.py
run r03h_bench 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0
run r03h_bench_dvc 300 python3 -u bench.py --config dvc --steps 10 --warmup 3 --cpu-baseline 0 --timer-steps 1
run r03h_bench_mm 300 python3 -u bench.py --config multimodal --steps 10 --warmup 3 --cpu-baseline 0
run r03h_bench_T4096 300 python3 -u bench.py --T 4096 --steps 10 --warmup 3 --cpu-baseline 0
run r03h_prof_dvc 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dvc -o run --output-format csv -- python3 bench.py --config dvc --steps 3 --warmup 2 --cpu-baseline 0 --timer-steps 0
run r03h_census 300 python3 -u tools/op_census.py
