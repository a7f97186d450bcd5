#!/bin/bash
# GPU call: k_tbatch A/B -- the winner's labels from LDS (KGPU_OPT_TBATCH_WLAB 1, default) against a global
# load (0), alternated, configs (c) / (d) at 5k and 100k; the 512 x 2 geometry (five workgroups at 5k
# nodes, KGPU_OPT_TBATCH_GEO 2) against the default 512 x 1; phase traces of the default.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_ab}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 300 python -u -m pytest tests/test_topo_persistent.py -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
B="--steps 10 --warmup 2 --cpu-sample 0 --latency-pods 0 --extras ''"
for w in c:5000 d:5000 c:100000 d:100000; do
  cfg=${w%%:*}; n=${w##*:}
  for r in 1 2; do
    for v in 1 0; do
      step ab_${cfg}${n}_wlab${v}_$r timeout -k 10 300 python3 -u bench.py --config $cfg --nodes $n --steps 10 --warmup 2 --cpu-sample 0 --latency-pods 0 --extras "" --tbatch-wlab $v || exit 1
    done
  done
done
for r in 1 2; do
  for g in 1 2; do
    step geo_c5000_g${g}_$r timeout -k 10 300 python3 -u bench.py --config c --nodes 5000 --steps 10 --warmup 2 --cpu-sample 0 --latency-pods 0 --extras "" --tbatch-geo $g || exit 1
  done
done
step trace_c timeout -k 10 300 python3 -u tools/phase_trace_topo.py --config c --nodes 5000 --pods 1000 || exit 1
step trace_d timeout -k 10 300 python3 -u tools/phase_trace_topo.py --config d --nodes 5000 --pods 1000 || exit 1
