#!/bin/bash
# GPU call (round 2, first): persistent-kernel phase trace at 5k / 100k nodes, then the bench lines of
# configs a-d at their BASELINE sizes with the full-workload CPU baseline (1 / 16 / all-core workers).
set -e
mkdir -p gpurun_out
T=${1:-p1}
timeout -k 10 300 python -u tools/phase_trace.py --nodes 5000 --pods 1000 > gpurun_out/phase_${T}_b5k.log 2>&1
timeout -k 10 300 python -u tools/phase_trace.py --nodes 100000 --pods 1000 > gpurun_out/phase_${T}_b100k.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_${T}_b.log 2>&1
timeout -k 10 300 python -u bench.py --config a --nodes 500 --steps 1 --pods-per-step 1000 > gpurun_out/bench_${T}_a.log 2>&1
timeout -k 10 400 python -u bench.py --config c > gpurun_out/bench_${T}_c.log 2>&1
timeout -k 10 400 python -u bench.py --config d > gpurun_out/bench_${T}_d.log 2>&1
