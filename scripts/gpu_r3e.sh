#!/bin/bash
# head light-poll + granules: fused-model tests, steady per-kernel table (bf16 only)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_convnet_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e/tests.log 2>&1 || exit $?
bash scripts/gpu_convnet_trace.sh r3e/trace > gpurun_out/r3e/trace_table.txt 2>&1 || exit $?
