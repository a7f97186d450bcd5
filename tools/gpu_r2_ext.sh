#!/bin/bash
# GPU call: extender tests, then rocprof stats + phase traces (tools/gpu_r2_prof.sh).
set -e
mkdir -p gpurun_out
T=${1:-r02}
timeout -k 10 300 python -u -m pytest tests/test_extender.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ext_$T.log 2>&1
./tools/gpu_r2_prof.sh $T
