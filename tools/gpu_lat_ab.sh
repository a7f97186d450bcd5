#!/bin/bash
# GPU call: kgpu_schedule_one latency A/B of two builds -- kubernetes-1_amd/kgpu/libkgpu_a.so (A, a side
# build: KGPU_LIB_PATH) against the in-tree libkgpu.so (B) -- alternated, after the given parity tests on B.
#   tools/gpu_lat_ab.sh <out-name> "<workloads cfg:nodes ...>" [pytest selection ...]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-lat_ab}
WL=${2:-b:5000}
shift; shift
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
if [ $# -gt 0 ]; then
  step pytest timeout -k 10 900 python -u -m pytest "$@" -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
fi
for w in $WL; do
  cfg=${w%%:*}; n=${w##*:}
  for r in 1 2; do
    KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_a.so step lat_${cfg}${n}_A_$r timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes $n --pods 300 || exit 1
    step lat_${cfg}${n}_B_$r timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes $n --pods 300 || exit 1
  done
done
