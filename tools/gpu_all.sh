#!/bin/bash
# One GPU call: gpu parity suite, bench for configs (b) 5k, (b) 100k, (c), (d), rocprof kernel stats
# of (b) and (c).  Each GPU step has its own time limit; the chain stops at the first failure.
set -e
mkdir -p gpurun_out
TAG=${1:-all}
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_${TAG}_b.log 2>&1
timeout -k 10 300 python -u bench.py --nodes 100000 --cpu-sample 100 > gpurun_out/bench_${TAG}_b100k.log 2>&1
timeout -k 10 300 python -u bench.py --config c --steps 5 --cpu-sample 100 > gpurun_out/bench_${TAG}_c.log 2>&1
timeout -k 10 300 python -u bench.py --config d --steps 5 --cpu-sample 100 > gpurun_out/bench_${TAG}_d.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_b -o run -- python3 $R/bench.py --cpu-sample 0 --steps 5 > $R/gpurun_out/prof_${TAG}_b.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_c -o run -- python3 $R/bench.py --config c --cpu-sample 0 --steps 2 > $R/gpurun_out/prof_${TAG}_c.log 2>&1
