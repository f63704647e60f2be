#!/bin/bash
# Final-tree kernel traces: ConvNet steady tables (plain / forced) and a rocprofv3 --stats summary of the plain step.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4final && mkdir -p $OUT
cd /tmp
for v in plain forced; do
  F=""; [ $v = forced ] && F="--force-collectives"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$v -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py $F --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { tail -20 $OUT/prof_$v.err; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof_$v -name "*kernel_trace.csv" | head -1) amp_s 128 > $OUT/steady_$v.txt && cut -c1-140 $OUT/steady_$v.txt
  rm -rf $OUT/prof_$v
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/stats.json 2> $OUT/stats.err || { tail -20 $OUT/stats.err; exit 1; }
S=$(find $OUT/stats -name "*kernel_stats.csv" | head -1); cp "$S" $OUT/kernel_stats.csv && cut -c1-160 $OUT/kernel_stats.csv | head -12
find $OUT/stats -name "*kernel_trace.csv" -delete
