#!/bin/bash
# GPU call: topology parity (fused + six-launch), then config (c)/(d) bench with the fused kernel.
set -e
mkdir -p gpurun_out
TAG=${1:-fu2}
timeout -k 10 300 python -u -m pytest tests/test_topology_parity.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 200 python -u bench.py --config c --steps 5 --cpu-sample 0 --topo-fused 1 > gpurun_out/bench_${TAG}_c.log 2>&1
timeout -k 10 200 python -u bench.py --config d --steps 5 --cpu-sample 0 --topo-fused 1 > gpurun_out/bench_${TAG}_d.log 2>&1
