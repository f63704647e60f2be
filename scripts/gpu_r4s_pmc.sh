#!/bin/bash
# PMC passes over the ConvNet step (eager, kernel per kernel): pass 1 LDS / MFMA / VALU
# counters, pass 2 memory (TCC fetch / write / hit / miss); per-kernel tables, raw data removed.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4s && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run_pass() {
  local tag=$1; shift
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/raw_$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 32 --warmup 16 --no-graph --epochs 0 --no-baseline --extra-dtypes "" > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -5 $OUT/bench_$tag.err; return 1; }
  python3 $GRAFT_REPO_ROOT/scripts/pmc_table.py $(find $OUT/raw_$tag -name "*counter_collection.csv" | head -1) > $OUT/table_$tag.txt && rm -rf $OUT/raw_$tag
}
run_pass lds SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
run_pass mem FETCH_SIZE WRITE_SIZE SQ_WAVES && cat $OUT/table_lds.txt $OUT/table_mem.txt | cut -c1-220
