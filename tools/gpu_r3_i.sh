#!/bin/bash
# Round 3: k_batch row waves take their candidate from the partials (no wait for the publish);
# wave-aggregated atomics in k_tbatch_init; query pools in one staged copy; diag rows zeroed by the
# kernels that write them.  GPU suite, smoke, bench + phase traces, kgpu_schedule_one latency for c / d,
# and a kernel + HIP API trace of the (c) latency run (ordinary launches: exits cleanly).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3i}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_gpu timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_b timeout -k 10 400 python -u bench.py || exit 1
step trace_b timeout -k 10 180 python -u tools/phase_trace.py || exit 1
step lat_c timeout -k 10 300 python -u bench.py --config c --steps 3 --cpu-sample 0 --extra-nodes 0 --latency-pods 300 || exit 1
step lat_d timeout -k 10 300 python -u bench.py --config d --steps 3 --cpu-sample 0 --extra-nodes 0 --latency-pods 300 || exit 1
step trace_c timeout -k 10 180 python -u tools/phase_trace_topo.py --config c || exit 1
cd /tmp
step lat_trace_c timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/lat_trace_c -o run \
  -- python3 -u $R/bench.py --config c --steps 1 --cpu-sample 0 --extra-nodes 0 --latency-pods 50 --no-coop || exit 1
