#!/bin/bash
# GPU call: the whole GPU suite, then the kgpu_schedule_one cycle timelines (c, d) and latencies
# (b, c, d) at 5k nodes.
#   tools/gpu_r4_cycle.sh <out-name>
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cycle}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step cyc_c timeout -k 10 180 python -u tools/cycle_trace.py --config c --nodes 5000 || exit 1
step cyc_d timeout -k 10 180 python -u tools/cycle_trace.py --config d --nodes 5000 || exit 1
step lat_b timeout -k 10 120 python -u tools/latency_probe.py --config b --nodes 5000 --pods 300 || exit 1
step lat_c timeout -k 10 120 python -u tools/latency_probe.py --config c --nodes 5000 --pods 300 || exit 1
step lat_d timeout -k 10 120 python -u tools/latency_probe.py --config d --nodes 5000 --pods 300 || exit 1
