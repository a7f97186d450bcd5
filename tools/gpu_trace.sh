#!/bin/bash
# GPU call: persistent-kernel phase traces (config b) at several geometries.
set -e
mkdir -p gpurun_out
T=${1:-t1}
for g in 0 5 3; do
  timeout -k 10 120 python -u tools/phase_trace.py --nodes 5000 --pods 1000 --groups $g >> gpurun_out/trace_${T}.log 2>&1
done
timeout -k 10 120 python -u tools/phase_trace.py --nodes 100000 --pods 1000 >> gpurun_out/trace_${T}.log 2>&1
