#!/bin/bash
# igemm A/B on the conv shapes and the ResNet-50 step: channel-tile fill (DPA_IGEMM_FILL=0: always 128)
# and the two-register-set forward pipeline (DPA_IGEMM_PIPE=0: one set)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for cfg in "0 0" "512 0" "512 1"; do
  set -- $cfg
  tag=fill$1_pipe$2
  DPA_IGEMM_FILL=$1 DPA_IGEMM_PIPE=$2 timeout -k 10 240 python -u scripts/exp/conv_bench.py > gpurun_out/r3_conv_$tag.txt 2>&1 || exit $?
  DPA_IGEMM_FILL=$1 DPA_IGEMM_PIPE=$2 timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3_resnet_$tag.json 2> gpurun_out/r3_resnet_$tag.err || exit $?
done
