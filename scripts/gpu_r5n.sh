#!/bin/bash
# W>1 step shape on one GPU (--force-collectives): plain vs forced steady tables (bf16), fills
# captured into the step graphs, phase stamps plain / forced; fp32 bench with the slab sink.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && R=$PWD && OUT=$PWD/gpurun_out/${1:-r5n} && mkdir -p $OUT
timeout -k 10 200 python bench.py --amp-dtype fp32 --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" > $OUT/b32.json 2> $OUT/b32.err || { tail -5 $OUT/b32.err; exit 1; }
echo "fp32 $(grep -o '"ms_per_step": [0-9.]*' $OUT/b32.json | head -1)"
timeout -k 10 200 python scripts/exp/find_fill.py --force-collectives > $OUT/fill_forced.txt 2>&1 || { tail -5 $OUT/fill_forced.txt; exit 1; }
grep -A14 "^===" $OUT/fill_forced.txt | head -80; tail -1 $OUT/fill_forced.txt
timeout -k 10 200 python scripts/exp/find_fill.py --amp-dtype fp32 > $OUT/fill_fp32.txt 2>&1 || { tail -5 $OUT/fill_fp32.txt; exit 1; }
tail -1 $OUT/fill_fp32.txt
DPA_EXT_SO=ddp_practice_amd/_C_timing.so timeout -k 10 200 python scripts/stamp_step.py > $OUT/stamps_plain.txt 2>&1 || { tail -5 $OUT/stamps_plain.txt; exit 1; }
DPA_EXT_SO=ddp_practice_amd/_C_timing.so timeout -k 10 200 python scripts/stamp_step.py --forced > $OUT/stamps_forced.txt 2>&1 || { tail -5 $OUT/stamps_forced.txt; exit 1; }
cut -c1-200 $OUT/stamps_plain.txt $OUT/stamps_forced.txt
cd /tmp
for m in plain forced; do
  F=""; [ $m = forced ] && F="--force-collectives"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$m -o run -- \
    python3 $R/bench.py --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady $F > $OUT/prof_$m.json 2> $OUT/prof_$m.err || { tail -20 $OUT/prof_$m.err; exit 1; }
  python3 $R/scripts/trace_steady.py $(find $OUT/prof_$m -name "*kernel_trace.csv" | head -1) sgd 128 > $OUT/steady_$m.txt && cut -c1-150 $OUT/steady_$m.txt
  rm -rf $OUT/prof_$m
done
