#!/bin/bash
# The driver's multi-GPU launch form rehearsed on one GPU with the round-5 tree: torchrun,
# 2 and 4 ranks sharing the card (2: xGMI engine, fused DDP average + pre-checked AMP step;
# 4: the gated launch path), full bench incl. the 3-epoch phase; then the supervised form.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5t} && mkdir -p $OUT
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2957$n bench.py --gpus $n --steps 500 --warmup 32 --share-gpu > $OUT/cn_w$n.json 2> $OUT/cn_w$n.err || { tail -30 $OUT/cn_w$n.err; exit 1; }
  echo "torchrun W=$n: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"accuracy": [0-9.]*\|"comm_error": "[^"]*"\|"fallback": [a-z"]*\|"grad_avg": "[^"]*"' $OUT/cn_w$n.json | tr '\n' ' ')"
done
timeout -k 10 400 python bench.py --gpus 2 --share-gpu --steps 500 --warmup 32 > $OUT/cn_sup_w2.json 2> $OUT/cn_sup_w2.err || { tail -30 $OUT/cn_sup_w2.err; exit 1; }
echo "supervised W=2: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"accuracy": [0-9.]*\|"comm_error": "[^"]*"\|"fallback": [a-z"]*' $OUT/cn_sup_w2.json | tr '\n' ' ')"
