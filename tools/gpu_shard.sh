#!/bin/bash
# GPU call: gpu parity suite (incl. the sharded path), bench of the sharded path on a one-rank
# communicator at 5k / 125k nodes, default bench.
set -e
mkdir -p gpurun_out
TAG=${1:-sh}
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --shard --cpu-sample 0 > gpurun_out/bench_${TAG}_shard5k.log 2>&1
timeout -k 10 300 python -u bench.py --shard --nodes 125000 --cpu-sample 0 --steps 3 > gpurun_out/bench_${TAG}_shard125k.log 2>&1
timeout -k 10 300 python -u bench.py --cpu-sample 0 > gpurun_out/bench_${TAG}_b.log 2>&1
