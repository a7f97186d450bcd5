#!/bin/bash
# GPU call: schedule_one / arena / resident / abort suites, then cycle timelines and host traces.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-cyc2}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step cyc_c timeout -k 10 180 python -u tools/cycle_trace.py --config c --nodes 5000 || exit 1
for c in b c d; do
  step lat_$c env KGPU_HOST_TRACE=1 timeout -k 10 120 python -u tools/latency_probe.py --config $c --nodes 5000 --pods 300 || exit 1
done
