#!/bin/bash
# round 3: driver-style bench, full GPU test tier, then the igemm channel-tile fill A/B
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3c_gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r3c_gpu_tests.log
bash scripts/gpu_r3_conv.sh
