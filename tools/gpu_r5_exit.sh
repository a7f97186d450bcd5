#!/bin/bash
# GPU call: (1) the CPU baseline's scaling on the box's 16-CPU share, per phase (tools/cpu_scale.py,
# KGPU_REF_PHASES=1; no GPU); (2) the rocprofv3 exit fault without libkgpu or torch:
# tools/coop_exit_probe with an ordinary dispatch, then with hipLaunchCooperativeKernel (last: it may
# fault at exit, and nothing runs after it).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_exit
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
export KGPU_REF_PHASES=1
step cpu_b5k timeout -k 10 120 python3 $R/tools/cpu_scale.py b 5000 4000 1,2,4,8,12,15,16 || exit 1
step cpu_b100k timeout -k 10 200 python3 $R/tools/cpu_scale.py b 100000 200 1,4,8,16 || exit 1
step cpu_c5k timeout -k 10 120 python3 $R/tools/cpu_scale.py c 5000 1000 1,4,8,16 || exit 1
unset KGPU_REF_PHASES
step plain timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/plain -o run -- $R/tools/coop_exit_probe plain || exit 1
step coop timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/coop -o run -- $R/tools/coop_exit_probe coop
