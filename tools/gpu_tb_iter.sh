#!/bin/bash
# GPU call: k_tbatch iteration -- topology parity tests, bench lines for configs c/d, phase traces.
set -e
mkdir -p gpurun_out
T=${1:-tb}
O=gpurun_out/tb_$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_topo_persistent.py tests/test_full_size.py tests/test_abort.py > $O/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --config c --steps 10 --pods-per-step 1000 --cpu-sample 0 --latency-pods 0 > $O/bench_c.log 2>&1
timeout -k 10 300 python -u bench.py --config d --steps 10 --pods-per-step 1000 --cpu-sample 0 --latency-pods 0 > $O/bench_d.log 2>&1
timeout -k 10 120 python -u tools/phase_trace_topo.py --config c > $O/ttrace_c.log 2>&1
timeout -k 10 120 python -u tools/phase_trace_topo.py --config d > $O/ttrace_d.log 2>&1
