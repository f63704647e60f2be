#!/bin/bash
# Round-5 entry check: GPU tests, smoke, ConvNet bench, ResNet-50 bench + steady table +
# one step's launch sequence, per-shape conv benches.   bash scripts/gpu_r5a.sh TAG
set -o pipefail
TAG=${1:-r5a}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_native.json 2> $OUT/rn_native.err || { tail -20 $OUT/rn_native.err; exit 1; }
cat $OUT/rn_native.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 12 --warmup 3 > $OUT/rn_prof.json 2> $OUT/rn_prof.err || { tail -5 $OUT/rn_prof.err; exit 1; }
CSV=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $CSV amp_sgd_large 5 > $OUT/rn_steady.txt
python3 $GRAFT_REPO_ROOT/scripts/trace_seq.py $CSV amp_sgd_large > $OUT/rn_seq.txt
rm -rf $OUT/prof
head -3 $OUT/rn_steady.txt
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python scripts/exp/conv_bench.py > $OUT/conv_bench.txt 2>&1 || { tail -5 $OUT/conv_bench.txt; exit 1; }
tail -2 $OUT/conv_bench.txt
timeout -k 10 300 python scripts/exp/g1x1_bench.py > $OUT/g1x1_bench.txt 2>&1 || { tail -5 $OUT/g1x1_bench.txt; exit 1; }
grep network $OUT/g1x1_bench.txt
