#!/bin/bash
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-probe}
mkdir -p $O
cd $R && export TMPDIR=/tmp
KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/var/libkgpu_sstamp.so timeout -k 10 120 python -u tools/phase_trace_topo.py --config c --nodes 5000 --pods 1000 > $O/sstamp_c.log 2>&1 || exit 1
KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/var/libkgpu_sstamp.so timeout -k 10 120 python -u tools/phase_trace_topo.py --config d --nodes 5000 --pods 1000 > $O/sstamp_d.log 2>&1 || exit 1
