#!/bin/bash
# Round-5 re-run of round 4's stalled rehearsal (torchrun, 4 ranks sharing the one GPU,
# full bench incl. the 3-epoch phase) with the watchdog's exchange-state report, and the
# xGMI engine's state dump on a healthy 2-rank run.   bash scripts/gpu_r5g.sh TAG
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5g} && mkdir -p $OUT
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 4 --steps 500 --warmup 32 --share-gpu > $OUT/cn_w4.json 2> $OUT/cn_w4.err || { tail -30 $OUT/cn_w4.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"comm_error": "[^"]*"\|"fallback": [a-z]*' $OUT/cn_w4.json | head
grep '\[dpa watchdog\]' $OUT/cn_w4.err | head -8
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"steady_ms_per_step": [0-9.]*' $OUT/bench.json
