#!/bin/bash
# GPU call: drop-in latency A/B -- the side build libkgpu_c.so (KGPU_LIB_PATH) against the in-tree library,
# alternated, configs (b) (c) (d) at 5k nodes, after the schedule_one parity tests on the side build.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r06_latab}; mkdir -p $O; cd $R; export TMPDIR=/tmp
C=$R/kubernetes-1_amd/kgpu/libkgpu_c.so
KGPU_LIB_PATH=$C timeout -k 10 600 python -u -m pytest tests/test_schedule_one.py tests/test_abort.py tests/test_prepare_pods.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_c.log 2>&1 || exit 1
for r in 1 2; do for w in b c d; do
  KGPU_LIB_PATH=$C timeout -k 10 300 python3 -u tools/latency_probe.py --config $w --nodes 5000 --pods 300 > $O/lat_${w}_c_$r.log 2>&1 || exit 1
  timeout -k 10 300 python3 -u tools/latency_probe.py --config $w --nodes 5000 --pods 300 > $O/lat_${w}_base_$r.log 2>&1 || exit 1
done; done
