# GPU: full test tier + the three CLIs end to end (3 epochs, synthetic MNIST-shaped data)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-cli}
mkdir -p $OUT
timeout -k 10 500 python -m pytest tests -m gpu -q > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" $OUT/pytest.log | tail -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cd $OUT
timeout -k 10 300 python $GRAFT_REPO_ROOT/origin_main.py --gpu 0 --synthetic > origin.log 2>&1; echo "origin rc=$?"; cat origin.log | tail -4
timeout -k 10 300 python $GRAFT_REPO_ROOT/ddp_main.py --gpu 0 --synthetic > ddp.log 2>&1; echo "ddp rc=$?"; tail -4 ddp.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533 $GRAFT_REPO_ROOT/ddp_main_torchrun.py --gpu 0 --synthetic > torchrun.log 2>&1; echo "torchrun rc=$?"; tail -4 torchrun.log
