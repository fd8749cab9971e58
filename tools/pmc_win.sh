#!/bin/bash
# PMC passes over the row-block MFMA backward (tools/win_pmc_driver.py), one counter group per pass.
cd "${GRAFT_REPO_ROOT:-.}"; OUT=gpurun_out/pmcw${WIN_T:-1024}; mkdir -p $OUT; export TMPDIR=/tmp
run() { local name=$1; shift; rm -rf $OUT/$name
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- \
    python3 tools/win_pmc_driver.py > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU
run sq2 SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
run lds SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SMEM SQ_INST_LEVEL_LDS
python3 tools/pmc_summary.py $OUT > $OUT/summary.json; cat $OUT/summary.json
