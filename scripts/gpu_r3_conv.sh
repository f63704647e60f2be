#!/bin/bash
# igemm channel-tile fill A/B: conv shapes and the ResNet-50 step, DPA_IGEMM_FILL=0 (always 128) vs default
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for f in 0 512; do
  DPA_IGEMM_FILL=$f timeout -k 10 240 python -u scripts/exp/conv_bench.py > gpurun_out/r3_conv_fill$f.txt 2>&1 || exit $?
  DPA_IGEMM_FILL=$f timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3_resnet_fill$f.json 2> gpurun_out/r3_resnet_fill$f.err || exit $?
done
