#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dvc2 -o run --output-format csv -- python3 bench.py --config dvc --steps 12 --warmup 1 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r03k_prof_dvc.log 2>&1
rc=$?; echo "prof rc=$rc"; grep "^{" gpurun_out/r03k_prof_dvc.log | cut -c1-300; exit $rc
