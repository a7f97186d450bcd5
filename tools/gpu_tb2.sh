#!/bin/bash
set -e
mkdir -p gpurun_out
T=${1:-tb2}
timeout -k 10 600 python -u -m pytest tests/test_topo_persistent.py tests/test_topology_parity.py tests/test_persistent.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${T}.log 2>&1
timeout -k 10 120 python -u tools/phase_trace_topo.py --config c > gpurun_out/ttrace_${T}.log 2>&1
timeout -k 10 120 python -u tools/phase_trace_topo.py --config d >> gpurun_out/ttrace_${T}.log 2>&1
timeout -k 10 120 python -u tools/phase_trace.py --nodes 5000 --pods 1000 > gpurun_out/trace_${T}.log 2>&1
timeout -k 10 200 python -u bench.py --cpu-sample 0 --latency-pods 0 > gpurun_out/bench_${T}_b.log 2>&1
timeout -k 10 200 python -u bench.py --config c --cpu-sample 0 --latency-pods 0 > gpurun_out/bench_${T}_c.log 2>&1
timeout -k 10 200 python -u bench.py --config d --cpu-sample 0 --latency-pods 0 > gpurun_out/bench_${T}_d.log 2>&1
