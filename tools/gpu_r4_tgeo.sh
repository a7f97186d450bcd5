#!/bin/bash
# GPU call: the whole GPU suite (the 256-thread k_tbatch geometry is the default), then (c) / (d)
# bench lines at 5k nodes with geometry 0 (256 x 1) and 1 (512 x 1) alternating, and phase traces.
#   tools/gpu_r4_tgeo.sh <out-name>
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-tgeo}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
for k in 1 2; do
  for g in 0 1; do
    step bench_c_g${g}_$k timeout -k 10 200 python -u bench.py --config c --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 0 --tbatch-geo $g || exit 1
    step bench_d_g${g}_$k timeout -k 10 200 python -u bench.py --config d --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 0 --tbatch-geo $g || exit 1
  done
done
step trace_c timeout -k 10 120 python -u tools/phase_trace_topo.py --config c --nodes 5000 --pods 1000 || exit 1
step lat_c timeout -k 10 120 python -u tools/latency_probe.py --config c --nodes 5000 --pods 300 || exit 1
