# PMC counters for the bench kernels (usage: bash scripts/gpu_pmc.sh TAG "CTR1 CTR2 ..." [bench args])
set -o pipefail
TAG=${1:-pmc}; CTRS=${2:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"}; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 64 --warmup 16 "$@" > $OUT/bench.json 2> $OUT/bench.err
echo "pmc rc=$?"
