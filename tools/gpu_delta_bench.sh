#!/bin/bash
# GPU call: delta-stream cost at 100k nodes (tools/delta_bench.py) with rocprofv3 kernel stats.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_delta -o delta -- python3 -u tools/delta_bench.py --nodes 100000 --existing 100000 --reps 20 > gpurun_out/delta_bench.jsonl 2> gpurun_out/delta_bench.err
