#!/bin/bash
# PMC passes over the pair backward at the encoder shape, one counter group per pass
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pmcp; export TMPDIR=/tmp
ARGS=${MICRO_ARGS:-"--dtypes bf16 --regimes init --iters 3 --shapes enc --kernels fwd,bwd_all"}
run() { local name=$1; shift; rm -rf gpurun_out/pmcp/$name
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmcp/$name -o run --output-format csv -- \
    python3 tools/msda_microbench.py $ARGS > gpurun_out/pmcp/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run l2 TCC_HIT_sum TCC_MISS_sum
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU
run sq2 SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR
run ta TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
python3 tools/pmc_summary.py gpurun_out/pmcp > gpurun_out/pmcp/summary.json; cat gpurun_out/pmcp/summary.json
