#!/bin/bash
# GPU call: HBM traffic counters of the dominant kernel, one counter group per rocprofv3 pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for cfg in "b 5000" "b 100000"; do
  set -- $cfg
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/pmc_$1_$2_$ctr -o run -- python3 $R/bench.py --config $1 --nodes $2 --cpu-sample 0 --steps 2 > $R/gpurun_out/pmc_$1_$2_$ctr.log 2>&1
  done
done
