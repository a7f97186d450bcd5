#!/bin/bash
# Round 3 final validation: the whole GPU suite, smoke(), the default bench line (what the driver runs
# at round end) and the (c)/(d) lines with their kgpu_schedule_one latency.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3final}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_all timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_default timeout -k 10 600 python -u bench.py || exit 1
step bench_c timeout -k 10 400 python -u bench.py --config c --steps 3 --cpu-sample 0 --extra-nodes 0 --latency-pods 300 || exit 1
step bench_d timeout -k 10 400 python -u bench.py --config d --steps 3 --cpu-sample 0 --extra-nodes 0 --latency-pods 300 || exit 1
step trace_b timeout -k 10 180 python -u tools/phase_trace.py || exit 1
