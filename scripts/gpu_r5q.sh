#!/bin/bash
# Pre-checked AMP step (producer-side gradient checks, no grid barrier): GPU tests, bf16 A/B
# (DPA_PRECHECK=0 = the barrier), steady table.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && R=$PWD && OUT=$PWD/gpurun_out/${1:-r5q} && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_convnet_fused_gpu.py tests/test_ops_gpu.py tests/test_bench_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in new old; do
    E=""; [ $v = old ] && E="DPA_PRECHECK=0"
    env $E timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { tail -5 $OUT/b_${v}_$i.err; exit 1; }
    echo "bf16 $v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_${v}_$i.json | head -1)"
  done
done
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"steady_ms": [0-9.]*\|"value_fp32": [0-9.]*\|"value_fp16": [0-9.]*\|"accuracy": [0-9.]*' $OUT/bench.json
cd /tmp
for v in new old; do
  E=""; [ $v = old ] && E="DPA_PRECHECK=0"
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$v -o run -- \
    python3 $R/bench.py --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { tail -20 $OUT/prof_$v.err; exit 1; }
  python3 $R/scripts/trace_steady.py $(find $OUT/prof_$v -name "*kernel_trace.csv" | head -1) sgd 128 > $OUT/steady_$v.txt && cut -c1-150 $OUT/steady_$v.txt
  rm -rf $OUT/prof_$v
done
