#!/bin/bash
# Round-2 validation pass: new GPU tests first, then the whole GPU tier, then the bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_bench_gpu.py tests/test_cli_gpu.py \
  -v --timeout 120 --timeout-method thread --maxfail=4 > gpurun_out/r2a_new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -5 gpurun_out/r2a_new_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 2000 --warmup 50 --out gpurun_out/r2a_bench.jsonl \
  > gpurun_out/r2a_bench.log 2>&1
rc2=$?; echo "bench rc=$rc2"; tail -c 1500 gpurun_out/r2a_bench.log
exit $rc
