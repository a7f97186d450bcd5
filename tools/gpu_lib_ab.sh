#!/bin/bash
# GPU call: A/B of two builds of the library in one box -- kubernetes-1_amd/kgpu/libkgpu_a.so (A, a side
# build: KGPU_LIB_PATH) against the in-tree libkgpu.so (B) -- alternated bench runs of the given workloads,
# after the given parity tests on B.
#   tools/gpu_lib_ab.sh <out-name> "<workloads cfg:nodes ...>" [pytest selection ...]
#   TRACES="c:3 d:3": afterwards, k_tbatch phase traces of B (tools/phase_trace_topo.py --mode, 5k nodes)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-lib_ab}
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
  for r in 1 2 3; do
    KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_a.so step ab_${cfg}${n}_A_$r timeout -k 10 300 python3 -u bench.py --config $cfg --nodes $n --steps 20 --warmup 3 --cpu-sample 0 --latency-pods 0 --extras "" || exit 1
    step ab_${cfg}${n}_B_$r timeout -k 10 300 python3 -u bench.py --config $cfg --nodes $n --steps 20 --warmup 3 --cpu-sample 0 --latency-pods 0 --extras "" || exit 1
  done
done
for t in $TRACES; do
  cfg=${t%%:*}; m=${t##*:}
  step trace_${cfg}_m${m} timeout -k 10 300 python3 -u tools/phase_trace_topo.py --config $cfg --nodes 5000 --pods 1000 --mode $m || exit 1
done
