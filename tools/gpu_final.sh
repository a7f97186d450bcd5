#!/bin/bash
# GPU call: what the driver runs at round end -- gpu suite, smoke(), default bench.
set -e
mkdir -p gpurun_out
TAG=${1:-fin}
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config a --nodes 500 --steps 2 --pods-per-step 750 --cpu-sample 200 > gpurun_out/bench_${TAG}_a.log 2>&1
