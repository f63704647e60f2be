#!/bin/bash
# W=4 torchrun rehearsal (4 processes on one GPU) with one HIP hardware queue per process
# (GPU_MAX_HW_QUEUES=1): does the stall at the epoch-2 boundary go away?  Two runs.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5v} && mkdir -p $OUT
for i in 1 2; do
  GPU_MAX_HW_QUEUES=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 2958$i bench.py --gpus 4 --steps 500 --warmup 32 --share-gpu > $OUT/cn_w4_$i.json 2> $OUT/cn_w4_$i.err || { tail -30 $OUT/cn_w4_$i.err; exit 1; }
  echo "W=4 hwq1 run $i: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"accuracy": [0-9.]*\|"fallback": [a-z"]*' $OUT/cn_w4_$i.json | tr '\n' ' ')"
  grep -o '"comm_error": "[^"]*"' $OUT/cn_w4_$i.json | head -c 600; echo
done
