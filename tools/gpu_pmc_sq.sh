#!/bin/bash
# GPU call: SQ instruction / wait counters of the persistent kernels (one rocprofv3 --pmc pass each).
set -e
R=$GRAFT_REPO_ROOT
T=${1:-sq1}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for cfg in c b; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/pmc_${T}_$cfg -o run -- python3 $R/bench.py --config $cfg --cpu-sample 0 --latency-pods 0 --steps 2 > $R/gpurun_out/pmc_${T}_$cfg.log 2>&1
done
