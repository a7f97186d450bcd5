#!/bin/bash
# GPU call: config (b)'s phase trace with the in-tree library and with a side build whose stamp 5
# marks the row wave's own evaluation done before it waits for the helper waves.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-hbstamp}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step trace_b timeout -k 10 120 python -u tools/phase_trace.py --config b --nodes 5000 --pods 1000 || exit 1
step trace_b_var env KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/var/libkgpu_hbstamp.so timeout -k 10 120 python -u tools/phase_trace.py --config b --nodes 5000 --pods 1000 || exit 1
