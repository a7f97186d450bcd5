#!/bin/bash
# Round 3: reproduce the host SIGSEGV of tests/test_abort.py::test_abort_k_tbatch with the native
# backtrace (KGPU_SEGV_TRACE=1), then the rest of the suite only if it passes.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3dbg}
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
KGPU_SEGV_TRACE=1 step abort_tb timeout -k 10 300 python -u -m pytest tests/test_abort.py -x -v -m gpu -p no:faulthandler \
  --timeout 200 --timeout-method thread || exit 1
