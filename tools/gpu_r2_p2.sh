#!/bin/bash
# GPU call: the R2 (percentageOfNodesToScore) parity tests, then the round-2 probe.
set -e
mkdir -p gpurun_out
T=${1:-p2}
timeout -k 10 600 python -u -m pytest tests/test_percentage.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1
bash tools/gpu_r2_probe.sh $T
