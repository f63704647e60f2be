#!/bin/bash
# ResNet-50 step: round-2 igemm kernels (_C_r2igemm.so) vs this round's (pipe on / off), alternating, one run
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/r3i
R2=$PWD/ddp_practice_amd/_C_r2igemm.so
for i in 1 2; do
  DPA_EXT_SO=$R2 timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3i/r2_$i.json 2> gpurun_out/r3i/r2_$i.err || exit $?
  timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3i/pipe1_$i.json 2> gpurun_out/r3i/pipe1_$i.err || exit $?
  DPA_IGEMM_PIPE=0 timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3i/pipe0_$i.json 2> gpurun_out/r3i/pipe0_$i.err || exit $?
done
