#!/bin/bash
# Round 3: batch-ahead behind the per-pod boundary (kgpu/ahead.py): parity against per-pod cycles
# (tests/test_ahead.py), then the per-cycle cost with and without it (tools/ahead_bench.py).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3k}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_ahead timeout -k 10 400 python -u -m pytest tests/test_ahead.py tests/test_abi.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step ahead_b timeout -k 10 400 python -u tools/ahead_bench.py --config b --nodes 5000 --pods 2000 || exit 1
step ahead_c timeout -k 10 400 python -u tools/ahead_bench.py --config c --nodes 5000 --pods 1500 || exit 1
step ahead_d timeout -k 10 400 python -u tools/ahead_bench.py --config d --nodes 5000 --pods 1500 || exit 1
step bench_e125k timeout -k 10 600 python -u bench.py --config e --nodes 125000 --steps 3 --cpu-sample 200 --latency-pods 0 --extra-nodes 0 || exit 1
step lat_c_sixlaunch timeout -k 10 300 python -u bench.py --config c --steps 2 --cpu-sample 0 --extra-nodes 0 --latency-pods 300 --no-topo-persistent || exit 1
step lat_c_probe timeout -k 10 300 python -u tools/latency_probe.py --config c --pods 300 || exit 1
step lat_trace_c timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/lat_trace_c -o run \
  -- python -u tools/latency_probe.py --config c --pods 120 || exit 1
