#!/bin/bash
# GPU call: instruction-cache counters of the persistent topology kernel (one --pmc pass).
R=$GRAFT_REPO_ROOT
T=${1:-ic1}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 true
timeout -s KILL 90 rocprofv3 --pmc SQC_DCACHE_REQ SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/pmc_${T}_c -o run -- python3 $R/bench.py --config c --cpu-sample 0 --latency-pods 0 --steps 2 > $R/gpurun_out/pmc_${T}_c.log 2>&1
