#!/bin/bash
# GPU call: whole -m gpu suite, smoke(), the default bench line, rocprof kernel stats of config b.
set -e
mkdir -p gpurun_out
T=${1:-verify}
O=gpurun_out/ver_$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_b.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b -o run -- python3 -u bench.py --steps 5 --cpu-sample 0 --latency-pods 0 > $O/prof_b.log 2>&1
