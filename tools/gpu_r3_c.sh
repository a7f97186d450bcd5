#!/bin/bash
# Round 3, verification call: the round-3 device tests first (sharded topology, PTS state export,
# abort hooks, extender, preemption), then the whole -m gpu suite, smoke(), the default bench line;
# last, two rocprofv3 exit probes (the program leaving through os._exit, then the minimal HIP program
# with no torch and no libkgpu).  Each GPU step has its own limit; the first failure ends the call.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3c}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_new timeout -k 10 300 python -u -m pytest tests/test_xgmi_topology.py tests/test_pts_state_device.py \
  tests/test_abort.py tests/test_extender.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step pytest_gpu timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread \
  --durations=25 || exit 1
step smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_default timeout -k 10 400 python -u bench.py || exit 1
step trace_b timeout -k 10 180 python -u tools/phase_trace.py || exit 1
step trace_c timeout -k 10 180 python -u tools/phase_trace_topo.py --config c || exit 1
step trace_d timeout -k 10 180 python -u tools/phase_trace_topo.py --config d || exit 1
cd /tmp
step probe_osexit timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_osexit -o run \
  -- python3 -u $R/tools/exit_probe.py kgpu $O/maps_osexit.txt --os-exit || exit 1
step probe_min timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_min -o run \
  -- $R/tools/exit_probe_min
