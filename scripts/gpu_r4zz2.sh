#!/bin/bash
# ConvNet 4 ranks sharing the GPU: with and without the fused DDP gradient exchange in the
# AMP-SGD kernel (DPA_FUSED_GRAD=0 -> RCCL all-reduces), short runs, fast watchdog.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4zz2 && mkdir -p $OUT
export DPA_WATCHDOG_TIMEOUT=40 DPA_XGMI_TIMEOUT=8
for v in 0 1; do
  DPA_FUSED_GRAD=$v timeout -k 10 280 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 2957$v bench.py --gpus 4 --steps 200 --warmup 16 --epochs 0 --share-gpu --no-baseline --extra-dtypes "" > $OUT/cn_w4_fg$v.json 2> $OUT/cn_w4_fg$v.err
  echo "fused_grad=$v rc=$? $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"fallback": [a-z"]*' $OUT/cn_w4_fg$v.json | tr '\n' ' ') $(grep -o '"comm_error": "[^"]\{0,120\}' $OUT/cn_w4_fg$v.json)"
done
