#!/bin/bash
# Round 3: k_tbatch experiment build (KGPU_TB_EXP, libkgpu_exp.so: every statistics slot of a wave
# polled in one sweep, normalize quotients through ratio100) -- parity, then (c)/(d) against default.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3v}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
EXP="env KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_exp.so"
X="--steps 3 --cpu-sample 0 --extra-nodes 0 --latency-pods 0"
step pytest_exp $EXP timeout -k 10 900 python -u -m pytest tests/test_topo_persistent.py tests/test_topology_parity.py tests/test_soa_golden.py tests/test_pts_state_device.py tests/test_arena.py tests/test_full_size.py tests/test_abort.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step c_def timeout -k 10 300 python -u bench.py --config c $X || exit 1
step c_exp $EXP timeout -k 10 300 python -u bench.py --config c $X || exit 1
step d_def timeout -k 10 300 python -u bench.py --config d $X || exit 1
step d_exp $EXP timeout -k 10 300 python -u bench.py --config d $X || exit 1
step trace_c_exp $EXP timeout -k 10 180 python -u tools/phase_trace_topo.py --config c || exit 1
