#!/bin/bash
# GPU call: k_tbatch A/B -- a workgroup's own exchange granules from LDS (KGPU_OPT_TBATCH_OWN 1, default)
# against loading its own stores back (0), alternated, configs (c) / (d) at 5k and 100k; phase traces of
# the default.  The persistent-topology, resident-state and abort parity tests first.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_own}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests/test_run_all_filters.py tests/test_topo_persistent.py tests/test_topo_resident.py tests/test_abort.py tests/test_preemption.py tests/test_schedule_one.py tests/test_filter_reasons.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
for w in c:5000 d:5000 c:100000 d:100000; do
  cfg=${w%%:*}; n=${w##*:}
  for r in 1 2; do
    for v in 1 0; do
      step ab_${cfg}${n}_own${v}_$r timeout -k 10 300 python3 -u bench.py --config $cfg --nodes $n --steps 10 --warmup 2 --cpu-sample 0 --latency-pods 0 --extras "" --tbatch-own $v || exit 1
    done
  done
done
step trace_c timeout -k 10 300 python3 -u tools/phase_trace_topo.py --config c --nodes 5000 --pods 1000 || exit 1
step trace_d timeout -k 10 300 python3 -u tools/phase_trace_topo.py --config d --nodes 5000 --pods 1000 || exit 1
