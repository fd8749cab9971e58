set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_module.py tests/test_add_norm.py tests/test_dvc.py tests/test_train_step.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_mm.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --config multimodal --cpu-baseline 0 > gpurun_out/bench_mm.log 2>&1; echo "bench rc=$?"
