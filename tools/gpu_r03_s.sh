#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_seg_attention.py > gpurun_out/r03z_seg.log 2>&1
rc=$?; echo "seg rc=$rc"; tail -2 gpurun_out/r03z_seg.log; [ $rc -eq 0 ] || { grep -n "^E " gpurun_out/r03z_seg.log | head; exit $rc; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sa5 -o run --output-format csv -- python3 tools/seg_attn_microbench.py > gpurun_out/r03z_sa_prof.log 2>&1
rc=$?; echo "mb rc=$rc"; grep "fwd+bwd" gpurun_out/r03z_sa_prof.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config dvc --steps 20 --warmup 3 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r03z_bench_dvc.log 2>&1
rc=$?; echo "dvc bench rc=$rc"; tail -1 gpurun_out/r03z_bench_dvc.log | cut -c1-250
exit $rc
