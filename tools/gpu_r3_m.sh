#!/bin/bash
# Round 3: branch-light node evaluation (Least/Most reciprocal fast path without per-lane branches,
# scores on every lane of a wave with a feasible node).  eval microbenchmark old vs new, parity of the
# persistent and per-pod paths, then config (b) bench and phase trace.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3m}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step eval_old timeout -k 10 120 tools/eval_bench_old || exit 1
step eval_new timeout -k 10 120 tools/eval_bench || exit 1
step pytest_b timeout -k 10 900 python -u -m pytest tests/test_persistent.py tests/test_full_size.py tests/test_random_parity.py tests/test_schedule_one.py tests/test_abort.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step bench_b timeout -k 10 400 python -u bench.py || exit 1
step trace_b timeout -k 10 180 python -u tools/phase_trace.py || exit 1
step pytest_topo timeout -k 10 900 python -u -m pytest tests/test_topo_persistent.py tests/test_topology_parity.py tests/test_soa_golden.py tests/test_ahead.py tests/test_xgmi_topology.py tests/test_pts_state_device.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step lat_c_probe timeout -k 10 300 python -u tools/latency_probe.py --config c --pods 300 || exit 1
step bench_c timeout -k 10 400 python -u bench.py --config c --steps 3 --cpu-sample 0 --extra-nodes 0 --latency-pods 300 || exit 1
cd /tmp
step lat_trace_c timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/lat_trace_c -o run \
  -- python3 -u $R/bench.py --config c --steps 1 --cpu-sample 0 --extra-nodes 0 --latency-pods 120 --no-coop || exit 1
