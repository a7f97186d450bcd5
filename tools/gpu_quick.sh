#!/bin/bash
# GPU call: gpu tests, phase trace at 5k / 100k nodes, bench (5k persistent, 100k).
set -e
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 120 python -u tools/phase_trace.py > gpurun_out/phase_$TAG.log 2>&1
timeout -k 10 200 python -u tools/phase_trace.py --nodes 100000 >> gpurun_out/phase_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --nodes 100000 --cpu-sample 0 > gpurun_out/bench_${TAG}_100k.log 2>&1
