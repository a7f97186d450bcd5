#!/bin/bash
# GPU call: resident-state + topology suites, schedule_one latency (b/c/d) with host traces, and a
# kernel trace of the (d) latency probe (init / memset / k_tbatch durations per cycle).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-d1}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
for c in c d; do
  step lat_$c env KGPU_HOST_TRACE=1 timeout -k 10 120 python -u tools/latency_probe.py --config $c --nodes 5000 --pods 300 || exit 1
done
step prof_d timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof_d -o run -- python3 tools/latency_probe.py --config d --nodes 5000 --pods 300 || exit 1
