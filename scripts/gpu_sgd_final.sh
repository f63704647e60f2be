# Fused AMP-SGD default granules-per-lane: op tests, fused ConvNet + xGMI DDP tests, bench + trace
bash $GRAFT_REPO_ROOT/scripts/gpu_sgd_solo.sh ${1:-sgdf}
