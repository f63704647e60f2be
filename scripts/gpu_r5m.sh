#!/bin/bash
# fp32 plain fused SGD step (slab sums in the optimizer launch, fc wgrad in the conv2 wgrad
# launch): targeted GPU tests, fp32 A/B (DPA_PLAIN_FUSED=0), bf16 headline, fp32 steady table.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5m} && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_convnet_fused_gpu.py tests/test_xgmi_ddp_gpu.py tests/test_bench_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new old; do
    E=""; [ $v = old ] && E="DPA_PLAIN_FUSED=0"
    env $E timeout -k 10 200 python bench.py --amp-dtype fp32 --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" > $OUT/b32_${v}_$i.json 2> $OUT/b32_${v}_$i.err || { tail -5 $OUT/b32_${v}_$i.err; exit 1; }
    echo "fp32 $v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/b32_${v}_$i.json | head -1) $(grep -o '"accuracy": [0-9.]*' $OUT/b32_${v}_$i.json)"
  done
done
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"value_fp32": [0-9.]*\|"ms_per_step_fp32": [0-9.]*\|"accuracy": [0-9.]*' $OUT/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --amp-dtype fp32 --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) sgd 128 > $OUT/steady_fp32.txt && cut -c1-150 $OUT/steady_fp32.txt
rm -rf $OUT/prof
