#!/bin/bash
# GPU call: the whole -m gpu suite, smoke() and the default bench line (what the driver runs at round
# end), then the drop-in cycle's latency (KGPU_HOST_TRACE=1, configs b / c / d at 5k and 100k nodes), each
# step under its own time limit, stopping at the first failure.
#   tools/gpu_validate.sh <out-name> [pytest selection ...]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-validate}
shift
SEL=${@:-tests}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 1000 python -u -m pytest $SEL -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 || exit 1
export KGPU_HOST_TRACE=1
for w in b:5000 c:5000 d:5000 b:100000 c:100000 d:100000; do
  cfg=${w%%:*}; n=${w##*:}
  step lat_${cfg}${n} timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes $n --pods 300 || exit 1
done
