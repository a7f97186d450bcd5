#!/bin/bash
# Round 3: config (a) (default profile, 500 nodes) and (b) with the next query loaded early (default
# build) and late (KGPU_QN_LATE build, libkgpu_exp.so), alternating.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3s}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
X="--cpu-sample 0 --extra-nodes 0 --latency-pods 0"
for k in 1 2; do
step a_def_$k timeout -k 10 300 python -u bench.py --config a $X || exit 1
step a_late_$k env KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_exp.so timeout -k 10 300 python -u bench.py --config a $X || exit 1
done
step b_late env KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_exp.so timeout -k 10 300 python -u bench.py $X || exit 1
step b_def timeout -k 10 300 python -u bench.py $X || exit 1
