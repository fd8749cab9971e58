#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/op_attrib.py --config video --steps 2 --top 70 > gpurun_out/r04k_attrib_core.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/op_attrib.py --config dvc --steps 1 --top 90 > gpurun_out/r04k_attrib_dvc.log 2>&1
