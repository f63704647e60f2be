#!/bin/bash
# 64-wide wgrad swizzle fix: numerics, wgrad per-shape sweep, PMC (LDS conflicts), ResNet-50 bench
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2m && mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_conv_igemm_gpu.py tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u scripts/exp/conv_bench.py > $OUT/conv_bench.txt 2>&1 || { tail -20 $OUT/conv_bench.txt; exit 1; }
grep "network" $OUT/conv_bench.txt
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_$i.json 2> $OUT/rn_$i.err || { tail -20 $OUT/rn_$i.err; exit 1; }
  echo "run $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_$i.json)"
done
bash scripts/gpu_pmc.sh r3s2m_pmc "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_WAVE_CYCLES" --model resnet50 --steps 2 --warmup 1 --no-graph && \
python3 scripts/pmc_table.py $(find gpurun_out/r3s2m_pmc/prof -name "*counter_collection.csv" | head -1) > $OUT/pmc.txt && cut -c1-250 $OUT/pmc.txt | grep -E "kernel|wgrad"
rm -rf gpurun_out/r3s2m_pmc/prof
