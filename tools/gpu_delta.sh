#!/bin/bash
# GPU call: delta-stream parity tests, then the golden + persistent suites touched by the assume changes.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_delta.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/delta.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_soa_golden.py tests/test_persistent.py tests/test_topo_persistent.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/delta_regress.log 2>&1
