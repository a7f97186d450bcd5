#!/bin/bash
# Round 3: the 64-row-thread k_batch geometry (one row wave beside the communication wave) against
# 128 at configs (a) and (b); parity of every geometry; topology parity after the start-up loads change.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3n}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_geo timeout -k 10 600 python -u -m pytest tests/test_persistent.py tests/test_abort.py tests/test_xgmi.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step bench_b_geo1 timeout -k 10 300 python -u bench.py --batch-geo 1 --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
step bench_b_geo0 timeout -k 10 300 python -u bench.py --batch-geo 0 --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
step bench_b_geo1b timeout -k 10 300 python -u bench.py --batch-geo 1 --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
step bench_b_geo0b timeout -k 10 300 python -u bench.py --batch-geo 0 --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
step bench_a_geo1 timeout -k 10 300 python -u bench.py --config a --batch-geo 1 --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
step bench_a_geo0 timeout -k 10 300 python -u bench.py --config a --batch-geo 0 --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
step pytest_topo timeout -k 10 900 python -u -m pytest tests/test_topo_persistent.py tests/test_topology_parity.py tests/test_soa_golden.py tests/test_xgmi_topology.py tests/test_pts_state_device.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step lat_c_probe timeout -k 10 300 python -u tools/latency_probe.py --config c --pods 300 || exit 1
