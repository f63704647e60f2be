#!/bin/bash
# raw-barrier statistics epilogue, glds wgrad for 1x1, BN backward sums in the 1x1 dgrad epilogue:
# numerics, sweeps, ResNet-50 A/B, steady table
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2e && mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_resnet_gpu.py tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u scripts/exp/g1x1_bench.py > $OUT/g1x1_bench.txt 2>&1 || { tail -20 $OUT/g1x1_bench.txt; exit 1; }
grep "network total" $OUT/g1x1_bench.txt
timeout -k 10 300 python -u scripts/exp/conv_bench.py > $OUT/conv_bench.txt 2>&1 || { tail -20 $OUT/conv_bench.txt; exit 1; }
grep "network" $OUT/conv_bench.txt
for v in 1 0 1 0; do
  DPA_FUSE_BN_BWD=$v timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_f$v.json 2> $OUT/rn_f$v.err || { tail -20 $OUT/rn_f$v.err; exit 1; }
  echo "FUSE_BN_BWD=$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_f$v.json)"
done
DPA_STAT_DEFER_MIN=0 timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_defer0.json 2> $OUT/rn_defer0.err || { tail -20 $OUT/rn_defer0.err; exit 1; }
echo "DEFER_MIN=0 $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_defer0.json)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 12 --warmup 3 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -5 $OUT/prof_bench.err; exit 1; }
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) amp_sgd_large 5 > $OUT/steady.txt && cut -c1-150 $OUT/steady.txt | head -30
rm -rf $OUT/prof
