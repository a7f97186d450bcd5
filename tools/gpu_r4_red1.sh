#!/bin/bash
# GPU call: A/B of wg_partials with one wave max for both key variants (side build) against the
# in-tree library on config (b), alternating runs, then the side build's phase trace.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-red1}
V=$R/kubernetes-1_amd/kgpu/var/libkgpu_red1.so
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step par_var env KGPU_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread || exit 1
for r in 1 2 3; do
  step base_$r timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 || exit 1
  step var_$r env KGPU_LIB_PATH=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 || exit 1
done
step trace_var env KGPU_LIB_PATH=$V timeout -k 10 120 python -u tools/phase_trace.py --config b --nodes 5000 --pods 1000 || exit 1
step base_b100k timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --config b --nodes 100000 || exit 1
step var_b100k env KGPU_LIB_PATH=$V timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --config b --nodes 100000 || exit 1
