#!/bin/bash
# fp16 / fp32 ConvNet bench lines, the two-shot rehearsal timings (2 and 4 ranks on the
# one GPU) and the ResNet-50 2-rank shared-GPU rehearsal through DDP + SyncBN.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r2misc
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for dt in ${DTYPES-fp16 fp32}; do
  timeout -k 10 300 python bench.py --amp-dtype $dt --out $OUT/bench_$dt.jsonl > $OUT/bench_$dt.log 2>&1 || exit 1
  echo "$dt: $(grep -o '"value": [0-9.]*\|"vs_baseline": [0-9.]*\|"accuracy": [0-9.]*' $OUT/bench_$dt.jsonl | tr '\n' ' ')"
done
for w in 2 4; do
  timeout -k 10 240 python -u scripts/exp/xgmi_rehearsal.py $w > $OUT/twoshot_w$w.txt 2>&1 || { tail $OUT/twoshot_w$w.txt; exit 1; }
  cat $OUT/twoshot_w$w.txt | grep -v amdgpu
done
timeout -k 10 400 python bench.py --model resnet50 --gpus 2 --share-gpu --steps 10 --warmup 3 --out $OUT/rn_w2.jsonl > $OUT/rn_w2.log 2>&1 || { tail $OUT/rn_w2.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"comm": "[^"]*"' $OUT/rn_w2.jsonl
