# GPU test tier only (usage: bash scripts/gpu_test.sh TAG [pytest selection...])
set -o pipefail
TAG=${1:-test}; shift
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu "${@:-tests}" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -40
exit $rc
