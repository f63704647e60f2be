#!/bin/bash
# ConvNet head granule hand-off (batched re-poll): fused-model tests, bench, steady per-kernel table;
# ResNet-50 with the two-register-set pipeline on/off (one run)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/r3d
timeout -k 10 300 python -u -m pytest tests/test_convnet_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3d/tests.log 2>&1 || exit $?
bash scripts/gpu_convnet_trace.sh r3d/trace > gpurun_out/r3d/trace_table.txt 2>&1 || exit $?
for p in 0 1; do
  DPA_IGEMM_PIPE=$p timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3d/resnet_pipe$p.json 2> gpurun_out/r3d/resnet_pipe$p.err || exit $?
done
