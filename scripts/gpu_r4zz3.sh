#!/bin/bash
# The round-3 4-rank rehearsal command (self-launched supervisor, 1 epoch), then the 3-epoch
# torchrun form that stalled in r4zz, with a 40 s watchdog.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4zz3 && mkdir -p $OUT
export DPA_WATCHDOG_TIMEOUT=40
timeout -k 10 300 python -u bench.py --gpus 4 --share-gpu --steps 200 --warmup 20 --epochs 1 > $OUT/share4.json 2> $OUT/share4.err
echo "selflaunch epochs1 rc=$? $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"fallback": [a-z"]*' $OUT/share4.json | tr '\n' ' ')"
timeout -k 10 300 python -u bench.py --gpus 4 --share-gpu --steps 200 --warmup 20 > $OUT/share4_e3.json 2> $OUT/share4_e3.err
echo "selflaunch epochs3 rc=$? $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"fallback": [a-z"]*' $OUT/share4_e3.json | tr '\n' ' ')"
