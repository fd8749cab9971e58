#!/bin/bash
# Round evidence in one GPU session: PMC traffic of the MSDA kernels (copied to
# profiles/traffic_latest.json so the bench line carries it), bench (with cpu_baseline), rocprof
# kernel stats of the bench, the other bench lines (fp32, multimodal, T=4096, sparse, full DVC
# step) and the per-GEMM census.  Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
bash tools/pmc_msda.sh > gpurun_out/pmc.log 2>&1 || { echo "pmc failed"; tail -n 5 gpurun_out/pmc.log; exit 1; }
cp gpurun_out/pmc/traffic_latest.json profiles/traffic_latest.json && echo "pmc ok"
run bench 400 python3 -u bench.py --steps 20 --warmup 5
run rocprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0
run bench_fp32 400 python3 -u bench.py --steps 10 --warmup 3 --dtype fp32 --cpu-baseline 0
run bench_multimodal 400 python3 -u bench.py --steps 10 --warmup 3 --config multimodal --cpu-baseline 0
run bench_T4096 400 python3 -u bench.py --steps 10 --warmup 3 --T 4096 --cpu-baseline 0
run bench_sparse 400 python3 -u bench.py --steps 5 --warmup 2 --config sparse --cpu-baseline 0
run bench_dvc 400 python3 -u bench.py --steps 20 --warmup 3 --config dvc --cpu-baseline 0
run gemm_census 300 python3 -u tools/gemm_census.py gpurun_out/gemm_census.csv
