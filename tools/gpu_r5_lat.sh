#!/bin/bash
# GPU call: where a kgpu_schedule_one cycle and a kgpu_schedule_batch call spend their host time
# (KGPU_HOST_TRACE=1: p50 / p99 per step and what holds the p99), configs b / c / d at 5k and 100k
# nodes, the spinning synchronize (KGPU_SYNC_SPIN=1) against the default, and config (b)'s batch calls.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_lat}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
export KGPU_HOST_TRACE=1
for cfg in b c d; do
  step lat_${cfg}5000 timeout -k 10 200 python3 -u tools/latency_probe.py --config $cfg --nodes 5000 --pods 400 || exit 1
done
KGPU_SYNC_SPIN=1 step lat_c5000_spin timeout -k 10 200 python3 -u tools/latency_probe.py --config c --nodes 5000 --pods 400 || exit 1
for cfg in b c d; do
  step lat_${cfg}100000 timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes 100000 --pods 300 || exit 1
done
step batch_b5000 timeout -k 10 200 python3 -u bench.py --config b --steps 20 --warmup 3 --cpu-sample 0 --latency-pods 0 --extras "" || exit 1
