#!/bin/bash
# PMC counters for the MSDA kernels in the microbenchmark (fp32, init regime).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
run() { # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc/$name -o run --output-format csv -- \
    python3 tools/msda_microbench.py --dtypes fp32 --regimes init --iters 3 ${MICRO_ARGS:-} > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD
run p2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_BRANCH
