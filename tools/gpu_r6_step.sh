#!/bin/bash
# GPU call (round 6): the stat_select reproducer, the whole -m gpu suite, then drop-in latency traces.
#   tools/gpu_r6_step.sh <out-name> [latency workloads cfg:nodes ...]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06_step}
shift
WL=${@:-d:5000 d:100000 c:5000}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step repro timeout -k 10 60 ./tools/repro/stat_select
step pytest timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
export KGPU_HOST_TRACE=1
for w in $WL; do
  cfg=${w%%:*}; n=${w##*:}
  step lat_${cfg}${n} timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes $n --pods 300 || exit 1
done
