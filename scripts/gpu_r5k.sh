#!/bin/bash
# ConvNet fp32 (BASELINE config 2) steady-state kernel table, and the bf16 one for reference.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5k} && mkdir -p $OUT
cd /tmp
for dt in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$dt -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --amp-dtype $dt --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof_$dt.json 2> $OUT/prof_$dt.err || { tail -20 $OUT/prof_$dt.err; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof_$dt -name "*kernel_trace.csv" | head -1) sgd 128 > $OUT/steady_$dt.txt && cut -c1-150 $OUT/steady_$dt.txt
  rm -rf $OUT/prof_$dt
done
