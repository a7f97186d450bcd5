#!/bin/bash
# Round 3: Balanced through the Markstein quotient from the rows' reciprocals (default build) against
# the IEEE division sequence (KGPU_IEEE_BALANCED build, libkgpu_exp.so); the whole GPU suite on the
# default build first.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3p}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_all timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
for k in 1 2; do
step bench_def_$k timeout -k 10 300 python -u bench.py --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
step bench_exp_$k env KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_exp.so timeout -k 10 300 python -u bench.py --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
done
step trace_def timeout -k 10 180 python -u tools/phase_trace.py || exit 1
