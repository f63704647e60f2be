#!/bin/bash
# KxK convs on the glds kernel (zero page for padding): numerics, per-shape sweep, ResNet-50 A/B
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2f && mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u scripts/exp/conv_bench.py > $OUT/conv_bench.txt 2>&1 || { tail -20 $OUT/conv_bench.txt; exit 1; }
head -9 $OUT/conv_bench.txt | cut -c1-120; grep "network" $OUT/conv_bench.txt
for v in 1 0 1 0; do
  DPA_G3X3=$v timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_g3_$v.json 2> $OUT/rn_g3_$v.err || { tail -20 $OUT/rn_g3_$v.err; exit 1; }
  echo "G3X3=$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_g3_$v.json)"
done
DPA_STAT_DEFER_MIN=0 timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_defer0.json 2> $OUT/rn_defer0.err || { tail -20 $OUT/rn_defer0.err; exit 1; }
echo "DEFER_MIN=0 $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_defer0.json)"
