#!/bin/bash
# GPU call: the -m gpu suite, the drop-in latency probes (tools/gpu_r5_lat.sh), and config (b)'s step
# with pipelined batches against synchronous ones, alternated.
R=$GRAFT_REPO_ROOT
N=${1:-r05_v}
O=$R/gpurun_out/$N
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
for r in 1 2; do
  step pipe_$r timeout -k 10 200 python3 -u bench.py --config b --steps 20 --warmup 5 --cpu-sample 0 --latency-pods 0 --extras "" || exit 1
  step sync_$r timeout -k 10 200 python3 -u bench.py --config b --steps 20 --warmup 5 --cpu-sample 0 --latency-pods 0 --extras "" --no-pipeline || exit 1
done
bash tools/gpu_r5_lat.sh ${N}_lat
