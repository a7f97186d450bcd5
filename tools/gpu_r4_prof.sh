#!/bin/bash
# Round 4 profiling call (the kernels of the round-end bench).  Persistent kernels through ordinary
# launches (--no-coop): a process that made a cooperative launch faults in the HIP runtime's exit
# handler after rocprofv3's finalization, so every profiled run exits cleanly.
#   kernel stats (k_batch b, k_tbatch c / d) at 5k and 100k nodes, PMC FETCH_SIZE / WRITE_SIZE each
#   (one counter per pass), and one kernel + HIP API trace of the kgpu_schedule_one latency run (c).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4prof}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
cd /tmp
B="--steps 5 --cpu-sample 0 --latency-pods 0 --no-coop"
for cfg in ${CFGS:-b c d}; do
  for n in 5000 100000; do
    step prof_${cfg}${n} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${cfg}${n} -o run \
      -- python3 -u $R/bench.py --config $cfg --nodes $n $B || exit 1
    for ctr in FETCH_SIZE WRITE_SIZE; do
      step pmc_${cfg}_${n}_${ctr} timeout -s KILL 200 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${cfg}_${n}_${ctr} -o run \
        -- python3 $R/bench.py --config $cfg --nodes $n --steps 2 --cpu-sample 0 --latency-pods 0 --no-coop || exit 1
    done
  done
done
step lat_trace_c timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/lat_trace_c -o run \
  -- python3 -u $R/bench.py --config c --steps 1 --cpu-sample 0 --latency-pods 50 --no-coop || exit 1
