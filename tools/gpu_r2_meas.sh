#!/bin/bash
# GPU call: round-2 measurements -- bench lines for configs a/b/c/d at 5k nodes (10k pods for c/d),
# b/c/d at 100k nodes, rocprof kernel stats for b/c/d, phase traces for k_batch and k_tbatch.
set -e
mkdir -p gpurun_out
T=${1:-r02}
O=gpurun_out/meas_$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $O/bench_b.log 2>&1
timeout -k 10 300 python -u bench.py --config a --nodes 500 --steps 2 --pods-per-step 500 > $O/bench_a.log 2>&1
timeout -k 10 300 python -u bench.py --config c --steps 10 --pods-per-step 1000 > $O/bench_c.log 2>&1
timeout -k 10 300 python -u bench.py --config d --steps 10 --pods-per-step 1000 > $O/bench_d.log 2>&1
timeout -k 10 400 python -u bench.py --nodes 100000 --steps 10 --pods-per-step 1000 --cpu-sample 1000 > $O/bench_b100k.log 2>&1
timeout -k 10 400 python -u bench.py --config c --nodes 100000 --steps 10 --pods-per-step 1000 --cpu-sample 200 > $O/bench_c100k.log 2>&1
timeout -k 10 500 python -u bench.py --config d --nodes 100000 --steps 10 --pods-per-step 1000 --cpu-sample 200 > $O/bench_d100k.log 2>&1
for c in b c d; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 -u bench.py --config $c --steps 5 --pods-per-step 1000 --cpu-sample 0 --latency-pods 0 > $O/prof_$c.log 2>&1
done
timeout -k 10 120 python -u tools/phase_trace.py --nodes 5000 --pods 1000 > $O/trace_b5k.log 2>&1
timeout -k 10 200 python -u tools/phase_trace.py --nodes 100000 --pods 1000 > $O/trace_b100k.log 2>&1
timeout -k 10 120 python -u tools/phase_trace_topo.py --config c > $O/ttrace_c.log 2>&1
timeout -k 10 120 python -u tools/phase_trace_topo.py --config d > $O/ttrace_d.log 2>&1
