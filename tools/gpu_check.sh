#!/bin/bash
# One GPU session: gpu tests -> smoke -> bench -> rocprofv3 kernel stats of the bench.
# Stops at the first crash / timeout (rc other than 0/1); test failures (rc 1) continue.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name" ; date +%T
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  if [ "$name" = smoke ] && [ $rc -ne 0 ]; then echo "STOP: smoke failed"; exit 1; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
  step pytest_gpu 480 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider
fi
if [ "$MODE" = micro ]; then
  step micro 300 python -u tools/msda_microbench.py ${MICRO_ARGS:-}
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python -u bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3}
  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0
  find gpurun_out/prof -name "*kernel_stats.csv" | head -3
fi
