#!/bin/bash
set -e
./tools/gpu_delta.sh
./tools/gpu_delta_bench.sh
