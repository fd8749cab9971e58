set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 env MSDA_HIP_LIB=$PWD/multimodal-feature-learning_amd/lib/libmsda_hip_phase.so python3 -u tools/msda_microbench.py --dtypes bf16 --regimes init --iters 1 --shapes enc --kernels bwd_value > gpurun_out/phase.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/msda_microbench.py --dtypes bf16 > gpurun_out/micro.log 2>&1 || exit $?
bash tools/pmc_msda.sh > gpurun_out/pmc.log 2>&1
