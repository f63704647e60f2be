#!/bin/bash
# Isolation A/B: conv2_fwd deferred pooled stores only (p1) vs p1 + conv1 deferred gather stores with the
# step-counter arrival issued behind the sample loads (new), alternating on one box.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4q && mkdir -p $OUT
B="--steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes"
for i in 1 2 3; do
  for v in p1 new; do
    E=""; [ $v != new ] && E="DPA_EXT_SO=$PWD/ddp_practice_amd/_C_$v.so DPA_ALLOW_STALE_EXT=1"
    env $E timeout -k 10 200 python -u bench.py $B "" > $OUT/p_${v}_$i.json 2> $OUT/p_${v}_$i.err || { tail -20 $OUT/p_${v}_$i.err; exit 1; }
    echo "run $i $v plain $(grep -o '"ms_per_step": [0-9.]*' $OUT/p_${v}_$i.json)"
  done
done
