#!/bin/bash
# GPU call: drop-in latency A/B of the side build libkgpu_a.so (KGPU_LIB_PATH) against the in-tree library,
# alternated, after the one-pod parity tests on the side build.  tools/gpu_r6_ticket_ab.sh <out> "<cfg:nodes ...>"
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r06_ticket}; mkdir -p $O; cd $R; export TMPDIR=/tmp
A=$R/kubernetes-1_amd/kgpu/libkgpu_a.so
KGPU_LIB_PATH=$A timeout -k 10 600 python -u -m pytest tests/test_schedule_one.py tests/test_full_size.py tests/test_percentage.py tests/test_filter_reasons.py tests/test_run_all_filters.py tests/test_soa_golden.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_a.log 2>&1 || exit 1
for r in 1 2; do for w in ${2:-b:100000 t:100000 b:5000}; do
  cfg=${w%%:*}; n=${w##*:}
  KGPU_LIB_PATH=$A timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes $n --pods 300 --per-pod-pools 1 > $O/lat_${cfg}${n}_a_$r.log 2>&1 || exit 1
  timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes $n --pods 300 --per-pod-pools 1 > $O/lat_${cfg}${n}_base_$r.log 2>&1 || exit 1
done; done
