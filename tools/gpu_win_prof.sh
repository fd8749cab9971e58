#!/bin/bash
# rocprofv3 kernel stats of the A/B script (prepass and main kernel of the row-block backward
# separately, against the pair kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/win_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/win_prof -o run -- python3 tools/win_ab.py > gpurun_out/win_prof.log 2>&1
rc=$?; tail -5 gpurun_out/win_prof.log
f=$(find gpurun_out/win_prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
exit $rc
