#!/bin/bash
# GPU call: A/B of the helper waves' one-pod-ahead scalar request loads (side build) against the
# in-tree library on config (b), alternating runs, then the side build's phase trace.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-hbpre}
V=$R/kubernetes-1_amd/kgpu/var/libkgpu_hbpre.so
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step par_var env KGPU_LIB_PATH=$V timeout -k 10 300 python -u -m pytest tests/test_batch_helper.py tests/test_persistent.py -x -q -m gpu --timeout 120 --timeout-method thread || exit 1
for r in 1 2 3; do
  step base_$r timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 || exit 1
  step var_$r env KGPU_LIB_PATH=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 || exit 1
done
step trace_var env KGPU_LIB_PATH=$V timeout -k 10 120 python -u tools/phase_trace.py --config b --nodes 5000 --pods 1000 || exit 1
