#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | grep -v "Warning\|run_backward" | tail -n 4 | cut -c1-700; if [ $rc -ne 0 ]; then exit $rc; fi; }
run r03j_tests 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_linear.py tests/test_gpu_dvc_step.py tests/test_dvc.py -m gpu
run r03j_gemm_ab 300 python3 -u tools/small_gemm_ab.py
grep "^{" gpurun_out/r03j_gemm_ab.log
run r03j_bench_dvc 300 python3 -u bench.py --config dvc --steps 10 --warmup 3 --cpu-baseline 0 --timer-steps 1
