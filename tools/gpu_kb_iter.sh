#!/bin/bash
# GPU call: k_batch iteration -- persistent-kernel parity tests, bench lines, phase traces.
set -e
mkdir -p gpurun_out
T=${1:-kb}
O=gpurun_out/kb_$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_persistent.py tests/test_abort.py tests/test_full_size.py tests/test_xgmi.py > $O/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --cpu-sample 0 --latency-pods 0 > $O/bench_b.log 2>&1
timeout -k 10 300 python -u bench.py --nodes 100000 --cpu-sample 0 --latency-pods 0 > $O/bench_b100k.log 2>&1
timeout -k 10 300 python -u bench.py --config a --nodes 500 --steps 2 --pods-per-step 500 --cpu-sample 0 --latency-pods 0 > $O/bench_a.log 2>&1
timeout -k 10 120 python -u tools/phase_trace.py --nodes 5000 --pods 1000 > $O/trace_b5k.log 2>&1
timeout -k 10 200 python -u tools/phase_trace.py --nodes 100000 --pods 1000 > $O/trace_b100k.log 2>&1
