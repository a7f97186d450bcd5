#!/bin/bash
# Round 3: one-sweep statistics poll for 65-256 workgroups (100k-node shards): parity through the
# bench's CPU sample (placements identical), against the previous build (libkgpu_exp.so).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3w}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
EXP="env KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_exp.so"
X="--nodes 100000 --steps 3 --extra-nodes 0 --latency-pods 0"
step c_new timeout -k 10 400 python -u bench.py --config c $X --cpu-sample 100 || exit 1
step c_old $EXP timeout -k 10 400 python -u bench.py --config c $X --cpu-sample 0 || exit 1
step d_new timeout -k 10 400 python -u bench.py --config d $X --cpu-sample 100 || exit 1
step d_old $EXP timeout -k 10 400 python -u bench.py --config d $X --cpu-sample 0 || exit 1
step pytest_topo timeout -k 10 600 python -u -m pytest tests/test_topo_persistent.py tests/test_full_size.py tests/test_abort.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
