#!/bin/bash
# GPU call: one-pod topology cycles -- side build libkgpu_a.so (k_tbatch's grouped leave counters) against the
# in-tree library, alternated, after the topology / one-pod / abort parity tests on the side build.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r06_leave}; mkdir -p $O; cd $R; export TMPDIR=/tmp
A=$R/kubernetes-1_amd/kgpu/libkgpu_a.so
KGPU_LIB_PATH=$A timeout -k 10 600 python -u -m pytest tests/test_schedule_one.py tests/test_topo_persistent.py tests/test_topo_resident.py tests/test_prepare_pods.py tests/test_abort.py tests/test_topology_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_a.log 2>&1 || exit 1
for r in 1 2; do for w in ${2:-c:100000 d:100000 c:5000}; do
  cfg=${w%%:*}; n=${w##*:}
  KGPU_LIB_PATH=$A timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes $n --pods 300 > $O/lat_${cfg}${n}_a_$r.log 2>&1 || exit 1
  timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes $n --pods 300 > $O/lat_${cfg}${n}_base_$r.log 2>&1 || exit 1
done; done
