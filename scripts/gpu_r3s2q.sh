#!/bin/bash
# ConvNet headline: steps per captured graph 16 (default) vs 32 / 64, same box
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2q && mkdir -p $OUT
for k in ${SPG_LIST:-16 32 64 16 32 64}; do
  timeout -k 10 200 python -u bench.py --steps 2000 --warmup 64 --epochs 0 --no-baseline --extra-dtypes "" --steps-per-graph $k > $OUT/spg_$k.json 2> $OUT/spg_$k.err || { tail -20 $OUT/spg_$k.err; exit 1; }
  echo "spg=$k $(grep -o '"ms_per_step": [0-9.]*' $OUT/spg_$k.json)"
done
