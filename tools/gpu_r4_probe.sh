#!/bin/bash
# GPU call: per-pod phase traces of k_batch (b) and k_tbatch (c, d) at 5k nodes, the topology
# kgpu_schedule_one latency at 5k, each under its own time limit, stopping at the first failure.
#   tools/gpu_r4_probe.sh <out-name> [lib path]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-probe}
mkdir -p $O
cd $R && export TMPDIR=/tmp
[ -n "$2" ] && export KGPU_LIB_PATH=$2
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step trace_b timeout -k 10 120 python -u tools/phase_trace.py --config b --nodes 5000 --pods 1000 || exit 1
step trace_c timeout -k 10 120 python -u tools/phase_trace_topo.py --config c --nodes 5000 --pods 1000 || exit 1
step trace_d timeout -k 10 120 python -u tools/phase_trace_topo.py --config d --nodes 5000 --pods 1000 || exit 1
step lat_c timeout -k 10 120 python -u tools/latency_probe.py --config c --nodes 5000 --pods 300 || exit 1
step lat_d timeout -k 10 120 python -u tools/latency_probe.py --config d --nodes 5000 --pods 300 || exit 1
