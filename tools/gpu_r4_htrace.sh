#!/bin/bash
# GPU call: kgpu_schedule_one latency with the host trace (KGPU_HOST_TRACE=1), configs (b), (c), (d).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-htrace}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
for c in b c d; do
  step lat_$c env KGPU_HOST_TRACE=1 KGPU_SYNC_SPIN=1 timeout -k 10 120 python -u tools/latency_probe.py --config $c --nodes 5000 --pods 300 || exit 1
done
