# PMC counter passes over the ConvNet bench (one counter set per rocprofv3 run) + per-kernel tables
set -o pipefail
TAG=${1:-pmcp}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for CTRS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 32 --warmup 16 --no-graph --epochs 0 --no-baseline > $OUT/bench$i.json 2> $OUT/bench$i.err
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  f=$(find $OUT/p$i -name "*counter_collection.csv" | head -1)
  python3 $GRAFT_REPO_ROOT/scripts/pmc_table.py $f > $OUT/table$i.txt && cat $OUT/table$i.txt
done
