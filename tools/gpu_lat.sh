#!/bin/bash
# GPU call: the whole -m gpu suite, then kgpu_schedule_one latency (plain and under a HIP API trace).
set -e
mkdir -p gpurun_out
T=${1:-lat}
O=gpurun_out/lat_$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u tools/latency_probe.py --pods 300 > $O/lat_b.log 2>&1
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_lat -o run -- python3 -u tools/latency_probe.py --pods 100 > $O/prof_lat.log 2>&1
