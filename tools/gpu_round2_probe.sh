set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --conv-find 1 > gpurun_out/bench_find.log 2>&1; echo "bench find rc=$?"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --conv-find 0 > gpurun_out/bench_nofind.log 2>&1; echo "bench nofind rc=$?"
