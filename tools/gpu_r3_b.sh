#!/bin/bash
# Round 3, profiling call.  rocprofv3 runs of a HIP program on this image fault in the HIP runtime's
# own exit handler after the tool's finalization (gpurun_out/r3a/probe_kgpu.log + maps_kgpu.txt:
# libc exit -> libamdhip64 -> libhsa-runtime64 -> a /dev/dri mapping).  First: does rocprofv3 still
# write its files when the program leaves through os._exit (no exit handlers)?  If so, the k_tbatch
# kernel stats and PMC passes for configs c / d at 5k / 100k nodes run that way.  Last, the minimal HIP
# program (no torch, no libkgpu) under rocprofv3: a fault there is the runtime's, not this repo's.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3b}
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pts_state_device.py tests/test_abort.py tests/test_extender.py tests/test_preemption.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || exit 1
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_osexit -o run -- python3 -u $R/tools/exit_probe.py kgpu $O/maps_osexit.txt --os-exit > $O/probe_osexit.log 2>&1
echo "probe_osexit rc=$?" > $O/status.txt
if [ -f $O/probe_osexit/run_kernel_stats.csv ]; then
  for cfg in c d; do
    for n in 5000 100000; do
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${cfg}${n} -o run -- python3 -u $R/bench.py --config $cfg --nodes $n --steps 5 --cpu-sample 0 --latency-pods 0 --extra-nodes 0 --os-exit > $O/prof_${cfg}${n}.log 2>&1
      rc=$?; echo "prof_${cfg}${n} rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${cfg}_${n}_${ctr} -o run -- python3 $R/bench.py --config $cfg --nodes $n --cpu-sample 0 --latency-pods 0 --steps 2 --extra-nodes 0 --os-exit > $O/pmc_${cfg}_${n}_${ctr}.log 2>&1
        rc=$?; echo "pmc_${cfg}_${n}_${ctr} rc=$rc" >> $O/status.txt; [ $rc -eq 0 ] || exit $rc
      done
    done
  done
fi
timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/probe_min -o run -- $R/tools/exit_probe_min > $O/probe_min.log 2>&1
