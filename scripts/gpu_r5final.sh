#!/bin/bash
# Round-5 validation of the tree: every GPU test, smoke, the driver's bench command (20 / 5)
# and the default bench, ResNet-50 native, steady tables (ConvNet plain + forced, ResNet-50).
#   bash scripts/gpu_r5final.sh TAG
set -o pipefail
TAG=${1:-r5final}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"steady_ms": [0-9.]*\|"value_fp16": [0-9.]*\|"value_fp32": [0-9.]*\|"wall_3epoch_s": [0-9.]*\|"accuracy": [0-9.]*' $OUT/bench_driver.json | tr '\n' ' '; echo
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"steady_ms": [0-9.]*' $OUT/bench.json | tr '\n' ' '; echo
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_native.json 2> $OUT/rn_native.err || { tail -20 $OUT/rn_native.err; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $OUT/rn_native.json | tr '\n' ' '; echo
cd /tmp && export TMPDIR=/tmp
for m in plain forced; do
  F=""; [ $m = forced ] && F="--force-collectives"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$m -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady $F > $OUT/prof_$m.json 2> $OUT/prof_$m.err || { tail -20 $OUT/prof_$m.err; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof_$m -name "*kernel_trace.csv" | head -1) sgd 128 > $OUT/cn_steady_$m.txt && head -3 $OUT/cn_steady_$m.txt
  rm -rf $OUT/prof_$m
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_rn -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 12 --warmup 3 > $OUT/rn_prof.json 2> $OUT/rn_prof.err || { tail -5 $OUT/rn_prof.err; exit 1; }
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof_rn -name "*kernel_trace.csv" | head -1) amp_sgd_large 5 > $OUT/rn_steady.txt && head -3 $OUT/rn_steady.txt
rm -rf $OUT/prof_rn
