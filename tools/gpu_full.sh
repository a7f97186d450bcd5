#!/bin/bash
# GPU call: the whole -m gpu suite (as the driver runs it), smoke(), then the full-size parity tests.
set -e
mkdir -p gpurun_out
T=${1:-full}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$T.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
