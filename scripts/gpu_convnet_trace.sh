# ConvNet bench + steady-state per-kernel durations (kernel trace, graph replay)
set -o pipefail
TAG=${1:-cntr}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err && grep -o '"ms_per_step": [0-9.]*' $OUT/bench.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 320 --warmup 32 --extra-dtypes "" --no-baseline --epochs 0 > $OUT/prof.json 2> $OUT/prof.err && \
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) amp_sgd 64 | cut -c1-130
