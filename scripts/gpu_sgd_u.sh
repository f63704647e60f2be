# A/B of the fused AMP-SGD granules-per-lane (DPA_SGD_U = 1, 2, 4): ConvNet bench each, then
# the fused-SGD GPU tests under the chosen setting
set -o pipefail
TAG=${1:-sgdu}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for u in 4 2 1 4 2 1; do
  DPA_SGD_U=$u timeout -k 10 200 python bench.py > $OUT/bench_u$u.json 2> $OUT/bench_u$u.err || { tail $OUT/bench_u$u.err; exit 1; }
  echo "U=$u $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_u$u.json)"
done
for u in 1 2; do
  DPA_SGD_U=$u timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py -k "fused_amp_sgd or scaler" > $OUT/tests_u$u.txt 2>&1 || { tail -30 $OUT/tests_u$u.txt; exit 1; }
  echo "U=$u tests: $(tail -1 $OUT/tests_u$u.txt)"
done
