#!/bin/bash
# Round 3: one-row-wave k_batch reads the variant-B candidate row across lanes (no LDS hand-off).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3r}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_b timeout -k 10 900 python -u -m pytest tests/test_persistent.py tests/test_abort.py tests/test_xgmi.py tests/test_full_size.py tests/test_random_parity.py tests/test_schedule_one.py tests/test_ahead.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
for k in 1 2; do
step bench_b_$k timeout -k 10 300 python -u bench.py --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
done
step bench_a timeout -k 10 300 python -u bench.py --config a --cpu-sample 0 --extra-nodes 0 --latency-pods 0 || exit 1
step trace_b timeout -k 10 180 python -u tools/phase_trace.py || exit 1
