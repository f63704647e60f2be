#!/bin/bash
# PMC passes over one conv shape (512 -> 512, 3x3, 7x7, bs 128: 196 workgroups, 72 K-steps)
# on the 4-wave (WIDE=0) and 8-wave (WIDE=4) kernels: where do the waves wait?
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5i} && mkdir -p $OUT
for wd in 0 4; do
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS" \
             "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
             "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/w${wd}_p$i -o run -- python3 scripts/exp/conv_one.py 512 7 512 3 1 30 $wd > $OUT/w${wd}_p$i.log 2>&1 || echo "pass $i w$wd failed"
    f=$(find $OUT/w${wd}_p$i -name "*counter_collection.csv" | head -1)
    [ -n "$f" ] && python3 scripts/pmc_table.py $f 2>/dev/null | grep -E "^kernel|conv_glds" > $OUT/w${wd}_p$i.txt; cat $OUT/w${wd}_p$i.txt
  done
done
