#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/dvc_graph_diag2.py > gpurun_out/r03m_diag.log 2>&1
rc=$?; echo "diag rc=$rc"; cat gpurun_out/r03m_diag.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config dvc --steps 20 --warmup 3 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r03m_bench_dvc.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r03m_bench_dvc.log | cut -c1-400
exit $rc
