#!/bin/bash
# 64-channel tiles for small grids (DPA_G1X1_BN64_BELOW): numerics, per-shape sweep, ResNet-50 A/B
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2k && mkdir -p $OUT
DPA_G1X1_BN64_BELOW=100000 timeout -k 10 400 python -u -m pytest tests/test_conv_igemm_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for b in 0 512 1024; do
  DPA_G1X1_BN64_BELOW=$b timeout -k 10 300 python -u scripts/exp/g1x1_bench.py > $OUT/g1x1_bench_b$b.txt 2>&1 || { tail -20 $OUT/g1x1_bench_b$b.txt; exit 1; }
  echo "BN64_BELOW=$b"; grep "network total" $OUT/g1x1_bench_b$b.txt
done
for b in 0 512 1024 0 512 1024; do
  DPA_G1X1_BN64_BELOW=$b timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_b$b.json 2> $OUT/rn_b$b.err || { tail -20 $OUT/rn_b$b.err; exit 1; }
  echo "BN64_BELOW=$b $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_b$b.json)"
done
