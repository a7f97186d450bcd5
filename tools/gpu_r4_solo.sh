#!/bin/bash
# GPU call: the solo statistics round of k_tbatch -- the whole GPU suite, phase traces of (c) and (d),
# bench lines with the ahead evaluation on / off, and a prefilter probe of a side-built stamp variant.
#   tools/gpu_r4_solo.sh <out-name>
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-solo}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step trace_c timeout -k 10 120 python -u tools/phase_trace_topo.py --config c --nodes 5000 --pods 1000 || exit 1
step trace_d timeout -k 10 120 python -u tools/phase_trace_topo.py --config d --nodes 5000 --pods 1000 || exit 1

for k in 1 2; do
  step bench_c$k timeout -k 10 200 python -u bench.py --config c --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 0 || exit 1
  step bench_cna$k timeout -k 10 200 python -u bench.py --config c --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 0 --topo-ahead 0 || exit 1
  step bench_d$k timeout -k 10 200 python -u bench.py --config d --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 0 || exit 1
done
