#!/bin/bash
# Round-end check in one GPU session: smoke, the whole GPU suite, then the evidence set
# (tools/gpu_evidence.sh: bench with cpu_baseline, rocprof, PMC, other bench lines, GEMM census).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; exit 1; }
echo "smoke ok"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
bash tools/gpu_evidence.sh
