#!/bin/bash
# GPU call: the -m gpu suite, then the drop-in latency probes with the host trace (tools/gpu_r5_lat.sh).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05_v}
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
bash tools/gpu_r5_lat.sh ${1:-r05_v}_lat
