#!/bin/bash
# --share-gpu now gives 3+ rank processes one HW queue each: CLI GPU tests, then the W=4
# torchrun rehearsal with the box's default environment (no GPU_MAX_HW_QUEUES override).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5w} && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_cli_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29591 bench.py --gpus 4 --steps 500 --warmup 32 --share-gpu > $OUT/cn_w4.json 2> $OUT/cn_w4.err || { tail -30 $OUT/cn_w4.err; exit 1; }
echo "torchrun W=4 (default env): $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"accuracy": [0-9.]*\|"fallback": [a-z"]*' $OUT/cn_w4.json | tr '\n' ' ')"
grep -o '"comm_error": "[^"]*"' $OUT/cn_w4.json | head -c 600; echo
