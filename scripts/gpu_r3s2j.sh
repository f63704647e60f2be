#!/bin/bash
# wgrad reduce (16 split groups per workgroup) numerics; wgrad split-target sweep on the ResNet-50 step
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2j && mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for b in 768 384 1536 768 512 1024; do
  DPA_WGRAD_BLOCKS=$b timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_b$b.json 2> $OUT/rn_b$b.err || { tail -20 $OUT/rn_b$b.err; exit 1; }
  echo "WGRAD_BLOCKS=$b $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_b$b.json)"
done
