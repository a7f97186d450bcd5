#!/bin/bash
# GPU call: alternated bench runs of up to three builds -- side builds libkgpu_a.so / libkgpu_b.so (KGPU_LIB_PATH)
# and the in-tree libkgpu.so -- on the given workloads, R rounds.
#   tools/gpu_ab3.sh <out-name> "<cfg:nodes ...>" [rounds]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab3}
WL=${2:-b:5000}
N=${3:-3}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
for w in $WL; do
  cfg=${w%%:*}; n=${w##*:}
  for r in $(seq 1 $N); do
    for v in a b base; do
      lib=$R/kubernetes-1_amd/kgpu/libkgpu_$v.so
      [ "$v" = base ] && lib=$R/kubernetes-1_amd/kgpu/libkgpu.so
      [ -f "$lib" ] || continue
      KGPU_LIB_PATH=$lib step ab_${cfg}${n}_${v}_$r timeout -k 10 300 python3 -u bench.py --config $cfg --nodes $n --steps 20 --warmup 3 --cpu-sample 0 --latency-pods 0 --dropin-pods 0 --extras "" || exit 1
    done
  done
done
