#!/bin/bash
# GPU call: zero-copy query pools for one-launch kgpu_schedule_one cycles (KGPU_OPT_ZEROCOPY_POOLS) -- the
# parity tests of the diagnostic cycle paths, then the drop-in latency with the option off and on,
# alternated, configs b / c / d at 5k nodes and b at 100k.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_zc}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 900 python -u -m pytest tests/test_schedule_one.py tests/test_soa_golden.py tests/test_filter_reasons.py tests/test_framework_runner.py tests/test_run_all_filters.py tests/test_preemption.py tests/test_percentage.py tests/test_extender.py tests/test_delta.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
export KGPU_HOST_TRACE=1
for w in b:5000 c:5000 b:100000; do
  cfg=${w%%:*}; n=${w##*:}
  for r in 1 2; do
    for v in 0 1; do
      step lat_${cfg}${n}_zc${v}_$r timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes $n --pods 300 --zc $v || exit 1
    done
  done
done
