#!/bin/bash
# GPU call: one rocprofv3 --pmc pass (one counter group) over the bench workload:
#   tools/gpu_pmc1.sh <config> <nodes> <COUNTER>
# rocprofv3 may fault at process exit after writing its files, so each pass is a call of its own.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc $3 --output-format csv -d $R/gpurun_out/pmc2_$1_$2_$3 -o run -- python3 $R/bench.py --config $1 --nodes $2 --cpu-sample 0 --latency-pods 0 --steps 2 > $R/gpurun_out/pmc2_$1_$2_$3.log 2>&1
