#!/bin/bash
# ResNet-50 (1 GPU, bs 128): steady-state per-kernel table from a kernel trace.
#   TAG=x bash scripts/gpu_resnet_steady.sh   -> gpurun_out/$TAG/steady.txt
set -o pipefail
TAG=${TAG:-rnsteady}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 12 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) amp_sgd_large 5 \
  > $OUT/steady.txt && cut -c1-150 $OUT/steady.txt | head -45
