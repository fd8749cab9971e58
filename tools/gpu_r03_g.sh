#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/dvc_graph_diag.py > gpurun_out/r03g_diag.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03g_diag.log | tail -32; [ $rc -eq 0 ] || exit $rc
DIAG_BF16=0 timeout -k 10 300 python3 -u tools/dvc_graph_diag.py > gpurun_out/r03g_diag32.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r03g_diag32.log | head -8; exit $rc
