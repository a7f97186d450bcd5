#!/bin/bash
# GPU call: k_batch helper waves -- the persistent / helper / full-size / abort suites, config (b)
# bench lines with the helpers on / off (alternating), and a phase trace.
#   tools/gpu_r4_hb2.sh <out-name>
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-hb2}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 600 python -u -m pytest tests/test_batch_helper.py tests/test_persistent.py tests/test_full_size.py tests/test_abort.py tests/test_schedule_one.py tests/test_ahead.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
for k in 1 2; do
  step bench_on$k timeout -k 10 200 python -u bench.py --config b --steps 20 --warmup 5 --cpu-sample 0 --latency-pods 0 --batch-helper 1 || exit 1
  step bench_off$k timeout -k 10 200 python -u bench.py --config b --steps 20 --warmup 5 --cpu-sample 0 --latency-pods 0 --batch-helper 0 || exit 1
done
step trace_b timeout -k 10 120 python -u tools/phase_trace.py --config b --nodes 5000 --pods 1000 || exit 1
