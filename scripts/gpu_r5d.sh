#!/bin/bash
# conv-kernel iteration: conv / ResNet GPU tests, ResNet-50 bench + steady table, A/B against
# DPA_WIDE=0 in the same call.   bash scripts/gpu_r5d.sh TAG
set -o pipefail
TAG=${1:-r5d}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_conv_igemm_gpu.py tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_new$i.json 2> $OUT/rn_new$i.err || { tail -20 $OUT/rn_new$i.err; exit 1; }
  DPA_WIDE=0 DPA_WGRAD_GLDS=1 DPA_WGRAD_WAVES=4 timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_old$i.json 2> $OUT/rn_old$i.err || { tail -20 $OUT/rn_old$i.err; exit 1; }
done
grep -o '"ms_per_step": [0-9.]*' $OUT/rn_*.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 12 --warmup 3 > $OUT/rn_prof.json 2> $OUT/rn_prof.err || { tail -5 $OUT/rn_prof.err; exit 1; }
CSV=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $CSV amp_sgd_large 5 > $OUT/rn_steady.txt
python3 $GRAFT_REPO_ROOT/scripts/trace_seq.py $CSV amp_sgd_large > $OUT/rn_seq.txt
rm -rf $OUT/prof
head -25 $OUT/rn_steady.txt | cut -c1-120
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_cli_gpu.py tests/test_dist_gpu.py > $OUT/pytest_cli.log 2>&1
rc=$?; echo "pytest cli rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $OUT/pytest_cli.log | tail -20
exit $rc
