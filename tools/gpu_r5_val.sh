#!/bin/bash
# GPU call: the -m gpu suite, smoke() and the default bench line (what the driver runs at round end),
# then the same default bench under rocprofv3 --kernel-trace --stats (every persistent launch is an
# ordinary dispatch since round 5: the run must exit cleanly).  Each step under its own time limit,
# stopping at the first failure.   tools/gpu_r5_val.sh <out-name> [pytest selection ...]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_val}
shift
SEL=${@:-tests}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest timeout -k 10 600 python -u -m pytest $SEL -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
step smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 || exit 1
cd /tmp
step prof timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-sample 0 --extra-cpu-sample 0 --latency-pods 50
