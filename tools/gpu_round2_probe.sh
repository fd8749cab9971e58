set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_sparse.py tests/test_train_step.py tests/test_dvc.py tests/test_dam.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_sparse.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --config sparse --cpu-baseline 0 > gpurun_out/bench_sparse.log 2>&1; echo "bench rc=$?"
