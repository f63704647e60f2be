#!/bin/bash
# fp32 conv2 backward with the weight-gradient launch on a forked side stream: ConvNet / ops /
# dist GPU tests, fp32 A/B (DPA_FP32_CONCURRENT=0 = one stream), fp32 steady table.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && R=$PWD && OUT=$PWD/gpurun_out/${1:-r5ab} && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_convnet_fused_gpu.py tests/test_ops_gpu.py tests/test_dist_gpu.py tests/test_xgmi_ddp_gpu.py tests/test_cli_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in conc serial; do
    E=""; [ $v = serial ] && E="DPA_FP32_CONCURRENT=0"
    env $E timeout -k 10 200 python bench.py --amp-dtype fp32 --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { tail -5 $OUT/b_${v}_$i.err; exit 1; }
    echo "fp32 $v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_${v}_$i.json | head -1)"
  done
done
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"value_fp16": [0-9.]*\|"value_fp32": [0-9.]*\|"accuracy": [0-9.]*' $OUT/bench_driver.json | tr '\n' ' '; echo
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $R/bench.py --amp-dtype fp32 --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python3 $R/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) sgd 128 > $OUT/steady_fp32.txt && cut -c1-150 $OUT/steady_fp32.txt
rm -rf $OUT/prof
