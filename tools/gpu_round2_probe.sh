set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_linear.py tests/test_gpu_glue.py tests/test_train_step.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_mods.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/bench2.log 2>&1; echo "bench rc=$?"
timeout -k 10 120 env MSDA_HIP_LIB=$PWD/multimodal-feature-learning_amd/lib/libmsda_hip_phase.so python3 -u tools/msda_microbench.py --dtypes bf16 --regimes init --iters 1 --shapes xmod,enc4096 --kernels bwd_all > gpurun_out/phase_x.log 2>&1; echo "phase rc=$?"
