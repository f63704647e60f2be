# Full validation: GPU tests, smoke, ConvNet bench, ResNet-50 bench, 2-rank shared-GPU ResNet DDP rehearsal
set -o pipefail
TAG=${1:-r2c_full}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_native.json 2> $OUT/rn_native.err || { tail -20 $OUT/rn_native.err; exit 1; }
cut -c1-200 $OUT/rn_native.json
timeout -k 10 400 python bench.py --model resnet50 --gpus 2 --share-gpu --steps 10 --warmup 3 > $OUT/rn_w2.json 2> $OUT/rn_w2.err || { tail -20 $OUT/rn_w2.err; exit 1; }
cut -c1-400 $OUT/rn_w2.json
