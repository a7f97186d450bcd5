#!/bin/bash
# GPU call: full gpu test suite, then configs (c) and (d) at 5000 nodes.
set -e
mkdir -p gpurun_out
TAG=${1:-t}
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config c --steps 5 --pods-per-step 1000 --cpu-sample 100 > gpurun_out/bench_${TAG}_c.log 2>&1
timeout -k 10 300 python -u bench.py --config d --steps 5 --pods-per-step 1000 --cpu-sample 100 > gpurun_out/bench_${TAG}_d.log 2>&1
