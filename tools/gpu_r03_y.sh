#!/bin/bash
# DVC step kernel trace of the final tree (per-step breakdown: tools/dvc_step_breakdown.py)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dvc_final -o run --output-format csv -- python3 bench.py --config dvc --steps 12 --warmup 2 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r03y_prof_dvc.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
