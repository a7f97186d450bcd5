#!/bin/bash
# Round 3 GPU call: the new sharded-topology test first (two ranks on one GPU, k_tbatch XG), then the
# whole -m gpu suite, smoke(), the default bench line, then ONE rocprofv3 exit probe (libkgpu.so only,
# no torch) that records /proc/self/maps, so the frames of a fault at process exit can be resolved.
# The probe runs last: a fault there ends the call.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3a}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_xgmi_topology.py -x -v --timeout 300 --timeout-method thread > $O/pytest_xtopo.log 2>&1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_b.log 2>&1
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_kgpu -o run -- python3 -u $R/tools/exit_probe.py kgpu $O/maps_kgpu.txt > $O/probe_kgpu.log 2>&1
