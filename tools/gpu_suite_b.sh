#!/bin/bash
# GPU call: the whole -m gpu suite, smoke(), the default bench line.
set -e
mkdir -p gpurun_out
T=${1:-sb}
O=gpurun_out/sb_$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_b.log 2>&1
