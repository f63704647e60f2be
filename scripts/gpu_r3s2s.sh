#!/bin/bash
# downsample BN inside bn3's residual apply: numerics, ResNet-50 A/B, 2-rank rehearsal
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2s && mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in 1 0 1 0; do
  DPA_FUSE_RBN_SUMS=$v timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_f$v.json 2> $OUT/rn_f$v.err || { tail -20 $OUT/rn_f$v.err; exit 1; }
  echo "run$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_f$v.json)"
done
timeout -k 10 400 python -u bench.py --model resnet50 --gpus 2 --share-gpu --steps 10 --warmup 3 > $OUT/rn_w2.json 2> $OUT/rn_w2.err || { tail -20 $OUT/rn_w2.err; exit 1; }
echo "w2 $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_w2.json) $(grep -o '"comm_error": "[^"]*"' $OUT/rn_w2.json)"
