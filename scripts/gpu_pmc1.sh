#!/bin/bash
# One PMC pass (LDS / MFMA counters) over the ConvNet bench (eager), per-kernel table.
set -o pipefail
TAG=${TAG:-pmc1}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -k 10 -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 32 --warmup 16 --no-graph --epochs 0 --no-baseline > $OUT/bench1.json 2> $OUT/bench1.err
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $GRAFT_REPO_ROOT/scripts/pmc_table.py $(find $OUT/p1 -name "*counter_collection.csv" | head -1) > $OUT/table1.txt
