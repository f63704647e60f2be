#!/bin/bash
# Final-tree sanity: smoke, ConvNet / ops GPU tests, the driver's bench command.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5sanity} && mkdir -p $OUT
timeout -k 10 200 python __graft_entry__.py > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_convnet_fused_gpu.py tests/test_ops_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"value_fp16": [0-9.]*\|"value_fp32": [0-9.]*\|"accuracy": [0-9.]*' $OUT/bench_driver.json | tr '\n' ' '; echo
