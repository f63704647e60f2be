# ResNet-50 iteration: GPU tests of the NHWC kernels + native bench + steady-state kernel trace
set -o pipefail
TAG=${1:-rnit}; BS=${2:-128}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model resnet50 --batch-size $BS --steps 20 --warmup 5 > $OUT/native.json 2> $OUT/native.err || { tail -20 $OUT/native.err; exit 1; }
cat $OUT/native.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --batch-size $BS --steps 8 --warmup 3 > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $f maxpool_fwd 5 > $OUT/steady.txt && head -45 $OUT/steady.txt
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --model resnet50 --batch-size $BS --steps 10 --warmup 3 --force-collectives > $OUT/forced.json 2> $OUT/forced.err || { tail -20 $OUT/forced.err; exit 1; }
cat $OUT/forced.json
