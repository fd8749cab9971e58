#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/small_gemm_ab.py > gpurun_out/r03j_gemm_ab.log 2>&1
rc=$?; grep "^{" gpurun_out/r03j_gemm_ab.log; exit $rc
