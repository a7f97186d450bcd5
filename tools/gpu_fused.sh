#!/bin/bash
# GPU call: parity suite (fused topology pipeline), then configs (c)/(d) bench and rocprof stats of (c).
set -e
mkdir -p gpurun_out
TAG=${1:-fu}
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py --config c --steps 5 --cpu-sample 100 > gpurun_out/bench_${TAG}_c.log 2>&1
timeout -k 10 300 python -u bench.py --config d --steps 5 --cpu-sample 100 > gpurun_out/bench_${TAG}_d.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_c -o run -- python3 $R/bench.py --config c --cpu-sample 0 --steps 2 > $R/gpurun_out/prof_${TAG}_c.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_d -o run -- python3 $R/bench.py --config d --cpu-sample 0 --steps 2 > $R/gpurun_out/prof_${TAG}_d.log 2>&1
