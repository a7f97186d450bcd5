#!/bin/bash
# GPU call: tools/own_probe.py (KGPU_OPT_TBATCH_OWN 0 / 1 placements against the C restatement); with
# _head/kubernetes-1_amd (a copy of another build's package) present, the same clusters on that build first
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_ownp}
mkdir -p $O
cd $R && export TMPDIR=/tmp
if [ -f _head/kubernetes-1_amd/kgpu/libkgpu.so ]; then
  timeout -k 10 600 python3 -u tools/own_probe.py none > $O/probe_head.log 2>&1
  echo "probe_head rc=$?" >> $O/status.txt
fi
timeout -k 10 600 python3 -u tools/own_probe.py 0 1 > $O/probe.log 2>&1; echo "probe rc=$?" >> $O/status.txt
