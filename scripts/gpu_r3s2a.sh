#!/bin/bash
# 1x1 glds GEMM kernel: numerics, per-shape sweep vs the general kernel and hipBLASLt, ResNet-50 A/B
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=gpurun_out/r3s2a && mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u scripts/exp/g1x1_bench.py > $OUT/g1x1_bench.txt 2>&1 || { tail -20 $OUT/g1x1_bench.txt; exit 1; }
cat $OUT/g1x1_bench.txt
for v in 1 0; do
  DPA_G1X1=$v timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_g1x1_$v.json 2> $OUT/rn_g1x1_$v.err || { tail -20 $OUT/rn_g1x1_$v.err; exit 1; }
  echo "DPA_G1X1=$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_g1x1_$v.json)"
done
