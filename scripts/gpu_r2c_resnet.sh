# ResNet-50 kernel-mode iteration: conv igemm + resnet GPU tests, native bench, steady-state trace
set -o pipefail
TAG=${1:-r2c_rn}; BS=${2:-128}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_conv_igemm_gpu.py tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed|Error" $OUT/pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model resnet50 --batch-size $BS --steps 20 --warmup 5 > $OUT/native.json 2> $OUT/native.err || { tail -20 $OUT/native.err; exit 1; }
cat $OUT/native.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --batch-size $BS --steps 12 --warmup 3 > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $f amp_sgd_large 5 > $OUT/steady.txt && cut -c1-150 $OUT/steady.txt | head -50
