set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_op.py tests/test_gpu_ops_api.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_op.log 2>&1; echo "tests rc=$?"
timeout -k 10 200 python3 -u tools/msda_microbench.py --dtypes bf16 --regimes init,trained --iters 50 --shapes enc,xmod,enc4096 --kernels bwd_all > gpurun_out/ab_new.log 2>&1; echo "micro rc=$?"
timeout -k 10 120 env MSDA_HIP_LIB=$PWD/multimodal-feature-learning_amd/lib/libmsda_hip_phase.so python3 -u tools/msda_microbench.py --dtypes bf16 --regimes init --iters 1 --shapes enc,enc4096 --kernels bwd_all > gpurun_out/phase_new.log 2>&1; echo "phase rc=$?"
