#!/bin/bash
# three-stage LDS-DMA conv pipeline: bitwise test, per-shape sweeps (2 vs 3 stages), ResNet-50 A/B
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2i && mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_igemm_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for st in 2 3; do
  DPA_GLDS_STAGES=$st timeout -k 10 300 python -u scripts/exp/g1x1_bench.py > $OUT/g1x1_bench_s$st.txt 2>&1 || { tail -20 $OUT/g1x1_bench_s$st.txt; exit 1; }
  DPA_GLDS_STAGES=$st timeout -k 10 300 python -u scripts/exp/conv_bench.py > $OUT/conv_bench_s$st.txt 2>&1 || { tail -20 $OUT/conv_bench_s$st.txt; exit 1; }
  echo "stages=$st"; grep "network total" $OUT/g1x1_bench_s$st.txt; grep "network forward" $OUT/conv_bench_s$st.txt
done
for st in 3 2 3 2; do
  DPA_GLDS_STAGES=$st timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_s$st.json 2> $OUT/rn_s$st.err || { tail -20 $OUT/rn_s$st.err; exit 1; }
  echo "stages=$st $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_s$st.json)"
done
