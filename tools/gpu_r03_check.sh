#!/bin/bash
# Round-3 check: the new parity tests (verbose, with their error reports), the whole GPU suite,
# then one bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bf16_composition.py \
  "tests/test_gpu_op.py::test_bf16_T4096_bench_instantiation_matches_oracle" \
  tests/test_gpu_op.py::test_striped_levels_near_lds_budget_take_workspace \
  tests/test_gpu_op.py::test_backward_without_required_workspace_is_refused \
  tests/test_gpu_glue.py > gpurun_out/r03_new_tests.log 2>&1
rc=$?; tail -n 30 gpurun_out/r03_new_tests.log; [ $rc -eq 0 ] || { echo "new tests rc=$rc"; exit $rc; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/r03_pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
rc=$?; cat gpurun_out/r03_bench.json | head -c 600; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py --config dvc --steps 10 --warmup 3 --timer-steps 1 > gpurun_out/r03_bench_dvc.json 2> gpurun_out/r03_bench_dvc.err
rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r03_bench_dvc.json')); print(d['value'], d['ms_per_step'], d.get('phases_ms_per_step'))"; exit $rc
