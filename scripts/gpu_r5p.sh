#!/bin/bash
# EXPERIMENT (upper bound): the fused AMP step without its grid barrier (DPA_AMP_NOBARRIER=1:
# per-workgroup non-finite decision, not the real semantics) vs with it, bf16 ConvNet.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5p} && mkdir -p $OUT
for i in 1 2 3; do
  for v in bar nobar; do
    E=""; [ $v = nobar ] && E="DPA_AMP_NOBARRIER=1"
    env $E timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { tail -5 $OUT/b_${v}_$i.err; exit 1; }
    echo "bf16 $v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_${v}_$i.json | head -1)"
  done
done
