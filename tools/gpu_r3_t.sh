#!/bin/bash
# Round 3: the short-cycle arena at every size (KGPU_OPT_ARENA_BYTES) against the C restatement.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3t}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
step pytest_arena timeout -k 10 600 python -u -m pytest tests/test_arena.py tests/test_schedule_one.py tests/test_abi.py -x -v -m gpu --timeout 300 --timeout-method thread || exit 1
