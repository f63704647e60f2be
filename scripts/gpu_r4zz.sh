#!/bin/bash
# Multi-rank rehearsals on the one GPU with this round's in-kernel exchanges: ResNet-50 with 2
# ranks (DDP + SyncBN through the statistics finishers' wide site, supervisor), the ConvNet with
# 2 and 4 ranks (driver-style torchrun launch).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4zz && mkdir -p $OUT
timeout -k 10 400 python -u bench.py --model resnet50 --gpus 2 --share-gpu --steps 10 --warmup 3 > $OUT/rn_w2.json 2> $OUT/rn_w2.err || { tail -20 $OUT/rn_w2.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"comm_error": "[^"]*"\|"xgmi[a-z_]*": "[^"]*"\|"fallback": [a-z]*' $OUT/rn_w2.json | head
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 1000 --warmup 64 --share-gpu > $OUT/cn_w2.json 2> $OUT/cn_w2.err || { tail -30 $OUT/cn_w2.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"comm_error": "[^"]*"\|"fallback": [a-z]*' $OUT/cn_w2.json | head
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 4 --steps 500 --warmup 32 --share-gpu > $OUT/cn_w4.json 2> $OUT/cn_w4.err || { tail -30 $OUT/cn_w4.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"comm_error": "[^"]*"\|"fallback": [a-z]*' $OUT/cn_w4.json | head
