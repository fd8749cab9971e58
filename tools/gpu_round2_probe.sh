set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_add_norm.py tests/test_gpu_linear.py tests/test_gpu_module.py tests/test_train_step.py tests/test_gpu_glue.py tests/test_dvc.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_mods.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bench2.log 2>&1; echo "bench rc=$?"
