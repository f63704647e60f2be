#!/bin/bash
# raw-barrier statistics epilogue (both conv kernels), glds wgrad for 1x1: numerics, sweeps, ResNet-50 A/B
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2d && mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u scripts/exp/g1x1_bench.py > $OUT/g1x1_bench.txt 2>&1 || { tail -20 $OUT/g1x1_bench.txt; exit 1; }
DPA_STAT_DEFER_MIN=0 timeout -k 10 300 python -u scripts/exp/g1x1_bench.py > $OUT/g1x1_bench_defer0.txt 2>&1 || { tail -20 $OUT/g1x1_bench_defer0.txt; exit 1; }
grep "network total" $OUT/g1x1_bench.txt $OUT/g1x1_bench_defer0.txt
timeout -k 10 300 python -u scripts/exp/conv_bench.py > $OUT/conv_bench.txt 2>&1 || { tail -20 $OUT/conv_bench.txt; exit 1; }
DPA_STAT_DEFER_MIN=0 timeout -k 10 300 python -u scripts/exp/conv_bench.py > $OUT/conv_bench_defer0.txt 2>&1 || { tail -20 $OUT/conv_bench_defer0.txt; exit 1; }
grep "network" $OUT/conv_bench.txt $OUT/conv_bench_defer0.txt
for d in 1024 0 1024 0; do
  DPA_STAT_DEFER_MIN=$d timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_d$d.json 2> $OUT/rn_d$d.err || { tail -20 $OUT/rn_d$d.err; exit 1; }
  echo "DEFER_MIN=$d $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_d$d.json)"
done
