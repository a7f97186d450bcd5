#!/bin/bash
# GPU call: persistent topology kernel first light -- topology parity tests, then c/d bench lines.
set -e
mkdir -p gpurun_out
T=${1:-tb1}
timeout -k 10 400 python -u -m pytest tests/test_topology_parity.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1
timeout -k 10 200 python -u bench.py --config c --cpu-sample 0 --latency-pods 0 > gpurun_out/bench_${T}_c.log 2>&1
timeout -k 10 200 python -u bench.py --config d --cpu-sample 0 --latency-pods 0 > gpurun_out/bench_${T}_d.log 2>&1
bash tools/gpu_trace.sh $T
