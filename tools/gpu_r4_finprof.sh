#!/bin/bash
# GPU call: rocprofv3 kernel statistics of the final tree's bench runs, configs (b) and (c) at 5k nodes.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-finprof}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step prof_b timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b -o run -- python3 bench.py --steps 20 --warmup 5 || exit 1
step prof_c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c -o run -- python3 bench.py --steps 10 --warmup 3 --config c || exit 1
