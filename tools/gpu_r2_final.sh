#!/bin/bash
# GPU call: the whole -m gpu suite, smoke(), bench lines for configs a/b/c/d (5k) and b/c/d (100k)
# with their CPU baselines, rocprof kernel stats for b at 5k and 100k (last: rocprofv3 may fault at
# process exit after writing its files).
set -e
mkdir -p gpurun_out
T=${1:-fin}
O=gpurun_out/fin_$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_b.log 2>&1
timeout -k 10 300 python -u bench.py --config a --nodes 500 --steps 2 --pods-per-step 500 > $O/bench_a.log 2>&1
timeout -k 10 300 python -u bench.py --config c --steps 10 --pods-per-step 1000 > $O/bench_c.log 2>&1
timeout -k 10 300 python -u bench.py --config d --steps 10 --pods-per-step 1000 > $O/bench_d.log 2>&1
timeout -k 10 400 python -u bench.py --nodes 100000 --steps 10 --pods-per-step 1000 --cpu-sample 1000 > $O/bench_b100k.log 2>&1
timeout -k 10 400 python -u bench.py --config c --nodes 100000 --steps 10 --pods-per-step 1000 --cpu-sample 200 > $O/bench_c100k.log 2>&1
timeout -k 10 500 python -u bench.py --config d --nodes 100000 --steps 10 --pods-per-step 1000 --cpu-sample 200 > $O/bench_d100k.log 2>&1
timeout -k 10 120 python -u tools/phase_trace.py --nodes 5000 --pods 1000 > $O/trace_b5k.log 2>&1
timeout -k 10 200 python -u tools/phase_trace.py --nodes 100000 --pods 1000 > $O/trace_b100k.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b -o run -- python3 -u bench.py --steps 5 --cpu-sample 0 --latency-pods 0 > $O/prof_b.log 2>&1
