#!/bin/bash
# Where the driver-style 20-step window's fixed cost goes: device span vs wall vs host issue
# time (DPA_BENCH_EVENTS=1), 20 / 5 and 2000 / 50 steps.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5y} && mkdir -p $OUT
for i in 1 2 3; do
  DPA_BENCH_EVENTS=1 timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-baseline --extra-dtypes "" --epochs 0 > $OUT/s_$i.json 2> $OUT/s_$i.err || { tail -5 $OUT/s_$i.err; exit 1; }
  grep "\[bench\]" $OUT/s_$i.err
done
DPA_BENCH_EVENTS=1 timeout -k 10 100 python bench.py --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/l.json 2> $OUT/l.err || { tail -5 $OUT/l.err; exit 1; }
grep "\[bench\]" $OUT/l.err
