# usage: bash scripts/gpu_rehearse4.sh TAG  (runs the xGMI GPU tests first)
# Multi-rank rehearsal on one GPU: ConvNet bench with 4 ranks sharing the card (xGMI engine,
# in-kernel SyncBN + gradient exchanges), ResNet-50 bench with 2 ranks sharing the card.
set -o pipefail
TAG=${1:-r4}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_xgmi_gpu.py tests/test_xgmi_ddp_gpu.py > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29571 bench.py --gpus 4 --steps 500 --warmup 64 --share-gpu > $OUT/share4.json 2> $OUT/share4.err || { tail -30 $OUT/share4.err; exit 1; }
cat $OUT/share4.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29572 bench.py --gpus 2 --steps 1000 --warmup 64 --share-gpu > $OUT/share2.json 2> $OUT/share2.err || { tail -30 $OUT/share2.err; exit 1; }
cat $OUT/share2.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29573 bench.py --gpus 2 --model resnet50 --steps 10 --warmup 3 --share-gpu > $OUT/rn_share2.json 2> $OUT/rn_share2.err || { tail -30 $OUT/rn_share2.err; exit 1; }
cat $OUT/rn_share2.json
