# GPU test tier, then the CLI phase timings (usage: bash scripts/gpu_tests_cli.sh TAG)
set -o pipefail
TAG=${1:-tc}
bash $GRAFT_REPO_ROOT/scripts/gpu_test.sh $TAG > /dev/null || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/$TAG/pytest.log
bash $GRAFT_REPO_ROOT/scripts/gpu_cli_phases.sh $TAG || exit 1
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc-per-node 1 ddp_main_torchrun.py --gpu 0 --synthetic > gpurun_out/$TAG/trun.log 2>&1 || exit 1
grep -E "Accuracy|elapsed" gpurun_out/$TAG/trun.log
