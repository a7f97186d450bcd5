#!/bin/bash
# GPU call (round-4 final): the whole -m gpu suite, smoke(), the default bench line and configs
# (c)/(d) at 5k and 100k nodes, schedule_one latency (b/c/d) with host traces, and a kernel trace of
# the (d) latency probe.  Each step under its own limit; stops at the first failure.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-final}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 || exit 1
step bench_b100k timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --config b --nodes 100000 || exit 1
for c in c d; do
  step bench_${c} timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --config $c || exit 1
  step bench_${c}100k timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --config $c --nodes 100000 || exit 1
done
for c in b c d; do
  step lat_$c env KGPU_HOST_TRACE=1 timeout -k 10 120 python -u tools/latency_probe.py --config $c --nodes 5000 --pods 300 || exit 1
done
step prof_d timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof_d -o run -- python3 tools/latency_probe.py --config d --nodes 5000 --pods 300 || exit 1
