# The three CLIs end to end on 1 GPU (3 epochs, synthetic MNIST-shaped data), with per-epoch metrics
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-cli}
mkdir -p $OUT && cd $OUT
timeout -k 10 300 python $GRAFT_REPO_ROOT/origin_main.py --gpu 0 --synthetic --metrics-file origin_metrics.jsonl > origin.log 2>&1 && tail -3 origin.log && \
timeout -k 10 300 python $GRAFT_REPO_ROOT/ddp_main.py --gpu 0 --synthetic --metrics-file ddp_metrics.jsonl > ddp.log 2>&1 && tail -3 ddp.log && \
timeout -k 10 300 python $GRAFT_REPO_ROOT/ddp_main.py --gpu 0 --synthetic --amp-dtype bf16 > ddp_bf16.log 2>&1 && tail -3 ddp_bf16.log && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533 $GRAFT_REPO_ROOT/ddp_main_torchrun.py --gpu 0 --synthetic > torchrun.log 2>&1 && tail -3 torchrun.log && \
cat origin_metrics.jsonl ddp_metrics.jsonl && ls -la *.pt
