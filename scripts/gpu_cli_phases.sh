# Where the CLI wall clock goes: phase times of origin_main / ddp_main (spawn) on 1 GPU, run twice
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-clip}
mkdir -p $OUT && cd $OUT
export DPA_PHASES=1
for i in 1 2; do
  timeout -k 10 300 python $GRAFT_REPO_ROOT/origin_main.py --gpu 0 --synthetic > origin$i.log 2>&1 && grep -E "phase|elapsed" origin$i.log && \
  timeout -k 10 300 python $GRAFT_REPO_ROOT/ddp_main.py --gpu 0 --synthetic > ddp$i.log 2>&1 && grep -E "phase|elapsed" ddp$i.log || exit 1
done
