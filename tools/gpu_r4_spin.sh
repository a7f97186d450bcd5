#!/bin/bash
# GPU call: kgpu_schedule_one latency with the default synchronize and with KGPU_SYNC_SPIN=1
# (alternating), configs (b) and (c) at 5k nodes, plus the geometry-256 parity test.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-spin}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_topo_persistent.py tests/test_schedule_one.py tests/test_arena.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
for k in 1 2; do
  step lat_b_def$k timeout -k 10 120 python -u tools/latency_probe.py --config b --nodes 5000 --pods 300 || exit 1
  step lat_b_spin$k env KGPU_SYNC_SPIN=1 timeout -k 10 120 python -u tools/latency_probe.py --config b --nodes 5000 --pods 300 || exit 1
  step lat_c_def$k timeout -k 10 120 python -u tools/latency_probe.py --config c --nodes 5000 --pods 300 || exit 1
  step lat_c_spin$k env KGPU_SYNC_SPIN=1 timeout -k 10 120 python -u tools/latency_probe.py --config c --nodes 5000 --pods 300 || exit 1
done
