#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_op.py tests/test_gpu_prologue.py tests/test_gpu_bf16_composition.py \
  -k "tiles or orders or row_block or T4096 or prologue or composition" > gpurun_out/r03f_tests.log 2>&1
rc=$?; tail -n 5 gpurun_out/r03f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/win_tiles_ab.py > gpurun_out/r03f_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03f_ab.log; [ $rc -eq 0 ] || exit $rc
WIN_SPLIT_AB=1 timeout -k 10 300 python3 -u tools/win_tiles_ab.py > gpurun_out/r03f_split.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03f_split.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/r03f_bench.json 2> gpurun_out/r03f_bench.err
rc=$?; head -c 300 gpurun_out/r03f_bench.json; echo; python3 -c "import json; d=json.load(open('gpurun_out/r03f_bench.json')); print(d['roofline']['all_msda'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dvc_step.py tests/test_dvc.py -m gpu > gpurun_out/r03f_dvc_tests.log 2>&1
rc=$?; tail -n 12 gpurun_out/r03f_dvc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config dvc --steps 10 --warmup 3 --cpu-baseline 0 --timer-steps 1 > gpurun_out/r03f_bench_dvc.json 2> gpurun_out/r03f_bench_dvc.err
rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r03f_bench_dvc.json')); print(d['value'], d['ms_per_step'], d.get('phases_ms_per_step'))"; tail -n 3 gpurun_out/r03f_bench_dvc.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dvc -o run --output-format csv -- python3 bench.py --config dvc --steps 3 --warmup 2 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r03f_prof_dvc.log 2>&1
rc=$?; echo "prof dvc rc=$rc"; exit $rc
