#!/bin/bash
# Run the MSDA microbenchmark against every variant build lib/libmsda_hip_<name>.so (tools
# only: MSDA_HIP_LIB selects the library), then the phase-timing build if present.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS=${MICRO_ARGS:-"--dtypes bf16 --regimes init,trained --kernels fwd,bwd_all"}
LIBDIR=multimodal-feature-learning_amd/lib
for lib in $LIBDIR/libmsda_hip.so $LIBDIR/libmsda_hip_*.so; do
  name=$(basename $lib .so)
  [ "$name" = libmsda_hip_phase ] && continue
  echo "== $name"
  timeout -k 10 200 env MSDA_HIP_LIB=$PWD/$lib python3 -u tools/msda_microbench.py $ARGS > gpurun_out/var_$name.log 2>&1 || exit $?
  grep '^{' gpurun_out/var_$name.log
done
if [ -f $LIBDIR/libmsda_hip_phase.so ]; then
  timeout -k 10 120 env MSDA_HIP_LIB=$PWD/$LIBDIR/libmsda_hip_phase.so python3 -u tools/msda_microbench.py \
    --dtypes bf16 --regimes init --iters 1 --kernels bwd_all > gpurun_out/var_phase.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/var_phase.log | tail -24
fi
