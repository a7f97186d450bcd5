#!/bin/bash
# Round 3: k_batch with the next pod's query issued before the evaluation (KGPU_QN_EARLY build,
# libkgpu_exp.so) against the default build (issued after the partials), both at 64 row threads.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3o}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_exp env KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_exp.so timeout -k 10 600 python -u -m pytest tests/test_persistent.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
for k in 1 2; do
step bench_def_$k timeout -k 10 300 python -u bench.py --batch-geo 0 --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
step bench_exp_$k env KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_exp.so timeout -k 10 300 python -u bench.py --batch-geo 0 --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
done
step trace_def timeout -k 10 180 python -u tools/phase_trace.py --batch-geo 0 || exit 1
step trace_exp env KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_exp.so timeout -k 10 180 python -u tools/phase_trace.py --batch-geo 0 || exit 1
