#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python3 -u tools/seg_attn_microbench.py > gpurun_out/r03r_sa.log 2>&1
rc=$?; echo "mb rc=$rc"; grep -v amdgpu.ids gpurun_out/r03r_sa.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sa -o run --output-format csv -- python3 tools/seg_attn_microbench.py > gpurun_out/r03r_sa_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
