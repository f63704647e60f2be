# Single-workgroup fused AMP-SGD: optimizer GPU tests, DDP xGMI tests, then bench + steady-state trace
set -o pipefail
TAG=${1:-solo}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ops_gpu.py tests/test_convnet_fused_gpu.py tests/test_xgmi_ddp_gpu.py > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -1 $OUT/tests.txt
bash scripts/gpu_convnet_trace.sh $TAG
