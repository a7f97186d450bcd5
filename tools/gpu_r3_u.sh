#!/bin/bash
# Round 3: k_tbatch statistics publish without per-slot divergent branches.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3u}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_topo timeout -k 10 900 python -u -m pytest tests/test_topo_persistent.py tests/test_topology_parity.py tests/test_soa_golden.py tests/test_xgmi_topology.py tests/test_pts_state_device.py tests/test_ahead.py tests/test_abort.py tests/test_arena.py tests/test_full_size.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step bench_c timeout -k 10 400 python -u bench.py --config c --steps 3 --cpu-sample 0 --extra-nodes 0 --latency-pods 200 || exit 1
step bench_d timeout -k 10 400 python -u bench.py --config d --steps 3 --cpu-sample 0 --extra-nodes 0 --latency-pods 200 || exit 1
step trace_c timeout -k 10 180 python -u tools/phase_trace_topo.py --config c || exit 1
step trace_d timeout -k 10 180 python -u tools/phase_trace_topo.py --config d || exit 1
