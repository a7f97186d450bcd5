#!/bin/bash
# GPU call: whole -m gpu suite, then the round-2 measurements (tools/gpu_r2_meas.sh).
set -e
mkdir -p gpurun_out
T=${1:-r02}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
./tools/gpu_r2_meas.sh $T
