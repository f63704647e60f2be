#!/bin/bash
# 1x1 kernel + shift prefetch + deferred stats + native fc: numerics, sweep, ResNet-50 A/B and steady table
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2c && mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_resnet_gpu.py tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u scripts/exp/g1x1_bench.py > $OUT/g1x1_bench.txt 2>&1 || { tail -20 $OUT/g1x1_bench.txt; exit 1; }
grep "network total" $OUT/g1x1_bench.txt
for v in 1 0; do
  DPA_G1X1=$v timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_g1x1_$v.json 2> $OUT/rn_g1x1_$v.err || { tail -20 $OUT/rn_g1x1_$v.err; exit 1; }
  echo "DPA_G1X1=$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_g1x1_$v.json)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 12 --warmup 3 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -5 $OUT/prof_bench.err; exit 1; }
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) amp_sgd_large 5 > $OUT/steady.txt && cut -c1-150 $OUT/steady.txt | head -45
rm -rf $OUT/prof
