# ConvNet iteration: fused-op GPU tests, bench (default and A/B env), steady-state kernel table
set -o pipefail
TAG=${1:-r2c_cn}; AB=${2:-DPA_SLAB_SCALAR=1}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_convnet_fused_gpu.py tests/test_ops_gpu.py > $OUT/pytest.log 2>&1 && tail -1 $OUT/pytest.log && \
timeout -k 10 200 python bench.py --no-baseline --epochs 0 --steps 4000 > $OUT/bench.json 2> $OUT/bench.err && grep -o '"ms_per_step": [0-9.]*' $OUT/bench.json && \
timeout -k 10 200 env $AB python bench.py --no-baseline --epochs 0 --steps 4000 > $OUT/bench_ab.json 2> $OUT/bench_ab.err && grep -o '"ms_per_step": [0-9.]*' $OUT/bench_ab.json && \
timeout -k 10 200 python bench.py --no-baseline --epochs 0 --steps 4000 > $OUT/bench2.json 2> $OUT/bench2.err && grep -o '"ms_per_step": [0-9.]*' $OUT/bench2.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 320 --warmup 32 --no-baseline --epochs 0 > $OUT/prof.json 2> $OUT/prof.err && \
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) amp_sgd 64 > $OUT/steady.txt && cut -c1-130 $OUT/steady.txt
