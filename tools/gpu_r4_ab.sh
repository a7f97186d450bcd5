#!/bin/bash
# GPU call: A/B of side-built kernel variants (tools/build_variant.sh) on configs (b), (c), (d) at 5k
# nodes: short bench lines per variant, alternating, each step under its own time limit.
#   tools/gpu_r4_ab.sh <out-name> <variant.so|cur> ...
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab}
shift
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
for rep in 1 2; do
  for v in "$@"; do
    tag=$(basename $v .so)
    D=$R
    if [ "$v" = cur ]; then unset KGPU_LIB_PATH
    elif [ -d "$R/$v" ]; then unset KGPU_LIB_PATH; D=$R/$v; tag=tree_$(basename $v)  # a whole other tree (git worktree)
    else export KGPU_LIB_PATH=$R/$v; fi
    cd $D
    step ${tag}_b$rep timeout -k 10 200 python -u bench.py --config b --steps 20 --warmup 5 --cpu-sample 0 --latency-pods 0 || exit 1
    step ${tag}_c$rep timeout -k 10 200 python -u bench.py --config c --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 0 || exit 1
    [ "$D" = "$R" ] && { step ${tag}_cna$rep timeout -k 10 200 python -u bench.py --config c --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 0 --topo-ahead 0 || exit 1; }
    step ${tag}_d$rep timeout -k 10 200 python -u bench.py --config d --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 0 || exit 1
    cd $R
  done
done
unset KGPU_LIB_PATH
