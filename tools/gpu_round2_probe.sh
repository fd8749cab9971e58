set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --timer-steps 0 > gpurun_out/rocprof.log 2>&1; echo "rocprof rc=$?"
