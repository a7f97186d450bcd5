#!/bin/bash
# Round 3: Markstein division / exact double Least in the register-resident rows, no scratch in k_tbatch;
# one-pod k_tbatch for kgpu_schedule_one (diagnostic topology cycles), RCCL loaded lazily,
# topology tables in one staged copy.  The GPU suite, schedule_one latency for configs c / d,
# per-workgroup phase traces of k_tbatch, then ONE rocprofv3 run of the kgpu probe with a normal exit
# (was: a fault in an exit handler after the tool's finalization) without any cooperative launch -- last,
# since it may fault.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3e}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_gpu timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_b timeout -k 10 400 python -u bench.py || exit 1
step trace_b timeout -k 10 180 python -u tools/phase_trace.py || exit 1
step lat_c timeout -k 10 300 python -u bench.py --config c --steps 3 --cpu-sample 0 --extra-nodes 0 --latency-pods 300 || exit 1
step lat_d timeout -k 10 300 python -u bench.py --config d --steps 3 --cpu-sample 0 --extra-nodes 0 --latency-pods 300 || exit 1
step trace_c timeout -k 10 180 python -u tools/phase_trace_topo.py --config c || exit 1
step trace_d timeout -k 10 180 python -u tools/phase_trace_topo.py --config d || exit 1
cd /tmp
step probe_kgpu timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_kgpu -o run \
  -- python3 -u $R/tools/exit_probe.py kgpu $O/maps_kgpu.txt --no-persistent
