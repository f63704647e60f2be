#!/bin/bash
# Fused-AMP grid-barrier state allocated at optimizer construction (no zero-fill node in the step graph):
# optimizer / ConvNet / CLI tests, bench, steady table.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4zi && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_convnet_fused_gpu.py tests/test_cli_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B="--steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes"
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py $B "" > $OUT/p_$i.json 2> $OUT/p_$i.err || { tail -20 $OUT/p_$i.err; exit 1; }
  timeout -k 10 200 python -u bench.py --force-collectives $B "" > $OUT/f_$i.json 2> $OUT/f_$i.err || { tail -20 $OUT/f_$i.err; exit 1; }
  echo "run $i plain $(grep -o '"ms_per_step": [0-9.]*' $OUT/p_$i.json) forced $(grep -o '"ms_per_step": [0-9.]*' $OUT/f_$i.json)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) amp_s 128 > $OUT/steady.txt && cut -c1-140 $OUT/steady.txt
rm -rf $OUT/prof
