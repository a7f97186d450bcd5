#!/bin/bash
# GPU call: the resident topology state (KGPU_OPT_TOPO_RESIDENT) -- its parity test and the
# schedule_one / arena / delta / topology suites it touches, then the cycle timelines and phase traces.
#   tools/gpu_r4_resident.sh <out-name>
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-resident}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step cyc_c timeout -k 10 180 python -u tools/cycle_trace.py --config c --nodes 5000 || exit 1
step cyc_d timeout -k 10 180 python -u tools/cycle_trace.py --config d --nodes 5000 || exit 1
step trace_b timeout -k 10 120 python -u tools/phase_trace.py --config b --nodes 5000 --pods 1000 || exit 1
step trace_c timeout -k 10 120 python -u tools/phase_trace_topo.py --config c --nodes 5000 --pods 1000 || exit 1
step trace_d timeout -k 10 120 python -u tools/phase_trace_topo.py --config d --nodes 5000 --pods 1000 || exit 1
for k in 1 2; do
  step bench_on$k timeout -k 10 200 python -u bench.py --config b --steps 20 --warmup 5 --cpu-sample 0 --latency-pods 0 --batch-helper 1 || exit 1
  step bench_off$k timeout -k 10 200 python -u bench.py --config b --steps 20 --warmup 5 --cpu-sample 0 --latency-pods 0 --batch-helper 0 || exit 1
done
for k in 1 2; do
  step bench_c_ahead$k timeout -k 10 200 python -u bench.py --config c --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 100 --topo-ahead 1 || exit 1
  step bench_c_noahead$k timeout -k 10 200 python -u bench.py --config c --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 0 --topo-ahead 0 || exit 1
done
step bench_d_ahead timeout -k 10 200 python -u bench.py --config d --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 100 --topo-ahead 1 || exit 1
step bench_d_noahead timeout -k 10 200 python -u bench.py --config d --steps 10 --warmup 3 --cpu-sample 0 --latency-pods 0 --topo-ahead 0 || exit 1
