#!/bin/bash
# Round 6 profiling call: the kernels of the round-end bench, every workload of its line (configs b, c, d
# at 5k and 100k nodes, and config (e)'s 125k-node shard): rocprofv3 kernel stats, then PMC FETCH_SIZE /
# WRITE_SIZE in passes of their own (tools/pmc_summary.py turns them into profiles/<tag>_pmc_traffic.json).
# Persistent kernels are ordinary launches (the default since round 5): every profiled run exits cleanly.
#   tools/gpu_r6_prof.sh <out-name>      (WORKLOADS="b:5000 ..." to choose)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r6prof}
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
cd /tmp
B="--steps 5 --warmup 1 --cpu-sample 0 --latency-pods 0 --extras ''"
for w in ${WORKLOADS:-b:5000 b:100000 c:5000 c:100000 d:5000 d:100000 e:125000}; do
  cfg=${w%%:*}; n=${w##*:}
  step prof_${cfg}${n} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${cfg}${n} -o run \
    -- python3 -u $R/bench.py --config $cfg --nodes $n --steps 5 --warmup 1 --cpu-sample 0 --latency-pods 0 --dropin-pods 0 --extras "" || exit 1
  for ctr in FETCH_SIZE WRITE_SIZE; do
    step pmc_${cfg}_${n}_${ctr} timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${cfg}_${n}_${ctr} -o run \
      -- python3 $R/bench.py --config $cfg --nodes $n --steps 2 --warmup 1 --cpu-sample 0 --latency-pods 0 --dropin-pods 0 --extras "" || exit 1
  done
done
