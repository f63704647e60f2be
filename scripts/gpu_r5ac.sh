#!/bin/bash
# Knobs re-checked now that the AMP step has no grid barrier: granules per lane of the fused
# step (DPA_SGD_U=1 default / 2) and the head's workgroup size (DPA_HEAD_NT=256 default / 1024).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5ac} && mkdir -p $OUT
for i in 1 2 3; do
  for v in base u2 nt1024; do
    E="DPA_BENCH_EVENTS=0"; [ $v = u2 ] && E="DPA_SGD_U=2"; [ $v = nt1024 ] && E="DPA_HEAD_NT=1024"
    env $E timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { tail -5 $OUT/b_${v}_$i.err; exit 1; }
    echo "bf16 $v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_${v}_$i.json | head -1)"
  done
done
