#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/dvc_graph_diag2.py > gpurun_out/r03i_diag.log 2>&1
rc=$?; grep -v "amdgpu.ids\|UserWarning\|run_backward" gpurun_out/r03i_diag.log | tail -30; exit $rc
