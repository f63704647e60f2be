#!/bin/bash
# One build->measure iteration on the GPU box:
#   1. the ConvNet GPU tests (+ any extra test files given in $TESTS)
#   2. bench.py (1 GPU, default steps)  -> gpurun_out/$TAG/bench.json
#   3. steady-state per-kernel table from a kernel trace -> gpurun_out/$TAG/steady.txt
# usage: TAG=r2b TESTS="tests/test_x.py" bash scripts/gpu_iter.sh
set -o pipefail
TAG=${TAG:-iter}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests/test_convnet_fused_gpu.py $TESTS -x -v --timeout 120 \
  --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --out $OUT/bench.jsonl > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"vs_baseline": [0-9.]*\|"wall_3epoch_s": [0-9.]*\|"accuracy": [0-9.]*' $OUT/bench.jsonl
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 320 --warmup 32 --epochs 0 --no-baseline > $OUT/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) amp_sgd 64 \
  > $OUT/steady.txt && cut -c1-140 $OUT/steady.txt
