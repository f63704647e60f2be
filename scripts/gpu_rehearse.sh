#!/bin/bash
# usage: bash scripts/gpu_rehearse.sh W TAG
# W ranks of bench.py sharing the ONE GPU of the box under torchrun (the driver's N-GPU launch
# shape; one HIP hardware queue and 1/W of the CUs per rank at 3+, runtime/device.py):
#   share_w${W}_host.json  --comm host: DDP / SyncBN collectives staged through gloo (no
#                        spinning kernel anywhere: the rank logic alone at world W)
#   share_w$W.json       default --share-gpu path: the xGMI engine, one launch per SyncBN
#                        collective at 3+ shared ranks (ops/convnet_fused._fused_site_engine)
#   share_w${W}_fused.json  batch 4, DPA_FUSED_SYNC=1 DPA_FUSED_GRAD=1: the in-kernel SyncBN
#                        sites and the AMP-SGD gradient exchange forced on (W rows, W-1 peers)
# Each JSON line must carry fallback null, comm_error "" and ranks_seen == W.
set -o pipefail
W=${1:-8}
TAG=${2:-rehearse$W}
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/$TAG && mkdir -p $OUT
run() {  # name, extra env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W \
    --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py --gpus $W --share-gpu --no-fallback \
    "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -40 $OUT/$name.err; return 1; }
  python - "$OUT/$name.json" "$W" <<'EOF'
import json, sys
rec = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
keys = ("value", "ms_per_step", "n_gpus", "ranks_seen", "fallback", "comm_error", "accuracy", "wall_3epoch_s")
print(sys.argv[1].rsplit("/", 1)[-1], {k: rec.get(k) for k in keys})
assert rec["ranks_seen"] == int(sys.argv[2]) and rec["fallback"] is None and not rec["comm_error"], rec
EOF
}
# the fused and default runs on a short synthetic set (64 / 16 steps per rank per epoch at batch 4 / 8):
# full 60k epochs of 8 ranks on one card stalled near their end (profiles/r6i_w8_fused_long_stall.txt)
SHORT="--train-samples $((W * 256)) --test-samples $((W * 64))"
run share_w${W}_host DPA_BENCH_WATCHDOG=60 -- --steps 300 --warmup 32 --no-baseline --no-steady --comm host --no-graph && \
run share_w${W}_fused DPA_FUSED_SYNC=1 DPA_FUSED_GRAD=1 DPA_BENCH_WATCHDOG=60 -- --steps 300 --warmup 32 \
  --batch-size 4 --no-baseline --no-steady $SHORT && \
run share_w$W DPA_BENCH_WATCHDOG=60 -- --steps 300 --warmup 32 --no-baseline --no-steady $SHORT
