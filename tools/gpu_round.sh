#!/bin/bash
# One GPU call: parity tests, bench (persistent and per-launch), rocprof kernel stats.  Each GPU
# step has its own time limit and the chain stops at the first failure.
set -e
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --no-persistent --cpu-sample 0 > gpurun_out/bench_${TAG}_launch.log 2>&1
timeout -k 10 300 python -u bench.py --nodes 100000 --cpu-sample 100 > gpurun_out/bench_${TAG}_100k.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-sample 0 --steps 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
