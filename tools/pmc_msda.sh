#!/bin/bash
# rocprofv3 PMC passes over the MSDA kernels at the bench's call shapes (bf16, B=8, init
# regime, level-major coordinates as the bench step runs them), one counter group per pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE do not
# fit one pass; no --pmc together with sys/runtime traces).  Summarised per kernel and grid
# by tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
ARGS=${MICRO_ARGS:-"--dtypes bf16 --regimes init --iters 3 --shapes enc --kernels fwd,bwd_all --layout level_major"}
run() { # name counters...
  local name=$1; shift
  rm -rf gpurun_out/pmc/$name
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc/$name -o run --output-format csv -- \
    python3 tools/msda_microbench.py $ARGS > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run l2 TCC_HIT_sum TCC_MISS_sum
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU
python3 tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc/traffic_latest.json > gpurun_out/pmc/summary.json &&
  cat gpurun_out/pmc/summary.json gpurun_out/pmc/traffic_latest.json
