set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for sr in 1073741824 100 64; do
timeout -k 10 120 env MSDA_HIP_STRIPED_ROWS=$sr python3 -u tools/msda_microbench.py --dtypes bf16 --regimes init,trained --iters 50 --shapes enc,xmod,enc4096 --kernels bwd_all > gpurun_out/ab_$sr.log 2>&1 || exit 1
timeout -k 10 120 env MSDA_HIP_STRIPED_ROWS=$sr MSDA_HIP_LIB=$PWD/multimodal-feature-learning_amd/lib/libmsda_hip_phase.so python3 -u tools/msda_microbench.py --dtypes bf16 --regimes init --iters 1 --shapes enc --kernels bwd_all > gpurun_out/phase_$sr.log 2>&1 || exit 1
done
