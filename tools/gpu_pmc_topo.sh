#!/bin/bash
# GPU call: HBM traffic counters of the topology pipeline (configs c, d at 5000 nodes), one
# counter per rocprofv3 pass.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in c d; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/pmc_${c}_5000_$ctr -o run -- python3 $R/bench.py --config $c --cpu-sample 0 --steps 1 --pods-per-step 500 > $R/gpurun_out/pmc_${c}_5000_$ctr.log 2>&1
  done
done
