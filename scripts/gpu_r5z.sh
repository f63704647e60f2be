#!/bin/bash
# Driver-style 20 / 5 window: one-step lead graph (default) vs none (DPA_BENCH_LEAD=0),
# 4 interleaved rounds, with the device span / host issue diagnostics.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5z} && mkdir -p $OUT
for i in 1 2 3 4; do
  for v in lead nolead; do
    E="DPA_BENCH_EVENTS=1"; [ $v = nolead ] && E="DPA_BENCH_EVENTS=1 DPA_BENCH_LEAD=0"
    env $E timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/s_${v}_$i.json 2> $OUT/s_${v}_$i.err || { tail -5 $OUT/s_${v}_$i.err; exit 1; }
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/s_${v}_$i.json) $(grep '\[bench\] 20' $OUT/s_${v}_$i.err)"
  done
done
