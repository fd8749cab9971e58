#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/op_census.py --config video --top 90 > gpurun_out/r04l_census_video.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/op_census.py --config dvc --top 140 > gpurun_out/r04l_census_dvc.log 2>&1
