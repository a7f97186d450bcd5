#!/bin/bash
# GPU call: rocprofv3 kernel stats for configs b/c/d, then k_batch / k_tbatch phase traces.
set -e
T=${1:-r02}
O=gpurun_out/meas_$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/phase_trace.py --nodes 5000 --pods 1000 > $O/trace_b5k.log 2>&1
timeout -k 10 200 python -u tools/phase_trace.py --nodes 100000 --pods 1000 > $O/trace_b100k.log 2>&1
timeout -k 10 120 python -u tools/phase_trace_topo.py --config c > $O/ttrace_c.log 2>&1
timeout -k 10 120 python -u tools/phase_trace_topo.py --config d > $O/ttrace_d.log 2>&1
for c in ${CONFIGS:-b c d}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 -u bench.py --config $c --steps 5 --pods-per-step 1000 --cpu-sample 0 --latency-pods 0 > $O/prof_$c.log 2>&1
done
