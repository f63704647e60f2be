# ConvNet kernel iteration: numerics tests of the fused op, bench, one PMC pass (LDS / MFMA)
set -o pipefail
TAG=${1:-cnit}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_convnet_fused_gpu.py tests/test_ops_gpu.py tests/test_dist_gpu.py > $OUT/pytest.log 2>&1 && tail -1 $OUT/pytest.log && \
timeout -k 10 200 python bench.py > $OUT/bench.json 2> $OUT/bench.err && cut -c1-200 $OUT/bench.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 32 --warmup 16 --no-graph > $OUT/pmc.json 2> $OUT/pmc.err && \
python3 $GRAFT_REPO_ROOT/scripts/pmc_table.py $(find $OUT/pmc -name "*counter_collection.csv" | head -1) > $OUT/pmc.txt && cat $OUT/pmc.txt
