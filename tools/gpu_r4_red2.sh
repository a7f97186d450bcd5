#!/bin/bash
# GPU call: the in-tree library (wg_partials with one wave max for both key variants) -- the whole
# -m gpu suite and smoke() -- then alternating config (b) runs against the previous build kept as a
# side library (var/libkgpu_base.so), and the in-tree phase trace.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-red2}
V=$R/kubernetes-1_amd/kgpu/var/libkgpu_base.so
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
for r in 1 2 3; do
  step base_$r env KGPU_LIB_PATH=$V timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 || exit 1
  step new_$r timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 || exit 1
done
step base_b100k env KGPU_LIB_PATH=$V timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --config b --nodes 100000 || exit 1
step new_b100k timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --config b --nodes 100000 || exit 1
step trace_new timeout -k 10 120 python -u tools/phase_trace.py --config b --nodes 5000 --pods 1000 || exit 1
