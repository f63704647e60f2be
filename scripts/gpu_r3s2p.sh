#!/bin/bash
# 2 ResNet-50 ranks sharing one GPU (DDP + SyncBN through the supervisor) with this round's kernels;
# distributed GPU tests
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2p && mkdir -p $OUT
timeout -k 10 400 python -u bench.py --model resnet50 --gpus 2 --share-gpu --steps 10 --warmup 3 > $OUT/rn_w2.json 2> $OUT/rn_w2.err || { tail -20 $OUT/rn_w2.err; exit 1; }
cut -c1-600 $OUT/rn_w2.json
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py tests/test_xgmi_gpu.py tests/test_xgmi_ddp_gpu.py tests/test_syncbn_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/dist_tests.log 2>&1 || { tail -30 $OUT/dist_tests.log; exit 1; }
tail -1 $OUT/dist_tests.log
