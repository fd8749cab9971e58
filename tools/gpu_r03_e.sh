#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/win_ab.py > gpurun_out/r03e_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03e_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03e_pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/r03e_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r03e_bench.json 2> gpurun_out/r03e_bench.err
rc=$?; head -c 200 gpurun_out/r03e_bench.json; echo; python3 -c "import json; d=json.load(open('gpurun_out/r03e_bench.json')); print(d['roofline'])"; exit $rc
