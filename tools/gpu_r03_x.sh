#!/bin/bash
# final-tree check: smoke + the whole GPU suite
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03x_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r03x_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03x_pytest_gpu.log 2>&1
rc=$?; tail -n 2 gpurun_out/r03x_pytest_gpu.log; exit $rc
