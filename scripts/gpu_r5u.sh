#!/bin/bash
# Host-side issue counts in the xGMI state report: dist GPU tests, then one more W=4 torchrun
# rehearsal on one GPU (4 processes sharing the card) -- if it stalls, the watchdog report
# now carries every rank's host-issued collective / site counts.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5u} && mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_dist_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29574 bench.py --gpus 4 --steps 500 --warmup 32 --share-gpu > $OUT/cn_w4.json 2> $OUT/cn_w4.err || { tail -30 $OUT/cn_w4.err; exit 1; }
echo "torchrun W=4: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"accuracy": [0-9.]*\|"fallback": [a-z"]*' $OUT/cn_w4.json | tr '\n' ' ')"
grep -o '"comm_error": "[^"]*"' $OUT/cn_w4.json | head -c 3000
