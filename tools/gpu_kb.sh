#!/bin/bash
# GPU call: k_batch iteration -- persistent parity tests, phase traces, config-b bench lines.
set -e
T=${1:-kb}
O=gpurun_out/kb_$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_persistent.py tests/test_full_size.py tests/test_abort.py tests/test_soa_golden.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 120 python -u tools/phase_trace.py --nodes 5000 --pods 1000 > $O/trace_b5k.log 2>&1
timeout -k 10 120 python -u tools/phase_trace.py --nodes 5000 --pods 1000 --groups 5 > $O/trace_b5k_g5.log 2>&1
timeout -k 10 200 python -u tools/phase_trace.py --nodes 100000 --pods 1000 > $O/trace_b100k.log 2>&1
timeout -k 10 200 python -u bench.py --cpu-sample 0 --latency-pods 0 > $O/bench_b.log 2>&1
timeout -k 10 300 python -u bench.py --nodes 100000 --cpu-sample 0 --latency-pods 0 > $O/bench_b100k.log 2>&1
