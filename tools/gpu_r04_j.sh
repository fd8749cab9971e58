#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/win_exp.py --regimes init --lq 577 --qorders 0 --exps 0,1,4,5,13 > gpurun_out/r04j_winexp_sparse.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04j_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r04j_prof_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04j_prof_dvc -o run --output-format csv -- python3 bench.py --config dvc --steps 6 --warmup 2 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r04j_prof_dvc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04j_prof_sparse -o run --output-format csv -- python3 bench.py --config sparse --steps 10 --warmup 2 --cpu-baseline 0 --timer-steps 0 > gpurun_out/r04j_prof_sparse.log 2>&1
