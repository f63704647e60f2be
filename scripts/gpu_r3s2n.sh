#!/bin/bash
# ConvNet conv2 image layout A/B: default (W+4, XOR swizzle) vs DPA_IMG_PAD8 (W+8, no swizzle)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2n && mkdir -p $OUT
P8=$PWD/ddp_practice_amd/_C_pad8.so
DPA_EXT_SO=$P8 timeout -k 10 300 python -u -m pytest tests/test_convnet_fused_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests_pad8.log 2>&1 || { tail -30 $OUT/tests_pad8.log; exit 1; }
tail -1 $OUT/tests_pad8.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > $OUT/def_$i.json 2> $OUT/def_$i.err || { tail -20 $OUT/def_$i.err; exit 1; }
  DPA_EXT_SO=$P8 timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > $OUT/pad8_$i.json 2> $OUT/pad8_$i.err || { tail -20 $OUT/pad8_$i.err; exit 1; }
  echo "default $(grep -o '"ms_per_step": [0-9.]*' $OUT/def_$i.json)  pad8 $(grep -o '"ms_per_step": [0-9.]*' $OUT/pad8_$i.json)"
done
cd /tmp
for v in def pad8; do
  if [ $v = pad8 ]; then export DPA_EXT_SO=$P8; else unset DPA_EXT_SO; fi
  timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --kernel-trace --stats --output-format csv -d $OUT/pmc_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 64 --warmup 16 --epochs 0 --no-baseline --extra-dtypes "" > $OUT/pmc_$v.json 2> $OUT/pmc_$v.err || { tail -5 $OUT/pmc_$v.err; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/pmc_table.py $(find $OUT/pmc_$v -name "*counter_collection.csv" | head -1) > $OUT/pmc_$v.txt && cut -c1-200 $OUT/pmc_$v.txt | grep -E "^kernel|conv5x5|conv2_bwd|head_step"
  rm -rf $OUT/pmc_$v
done
