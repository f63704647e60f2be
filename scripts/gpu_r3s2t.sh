#!/bin/bash
# max-pool backward with one index load per vector: pool tests, ResNet-50 bench + steady table
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r3s2t && mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_$i.json 2> $OUT/rn_$i.err || { tail -20 $OUT/rn_$i.err; exit 1; }
  echo "run $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_$i.json)"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --steps 12 --warmup 3 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -5 $OUT/prof_bench.err; exit 1; }
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) amp_sgd_large 5 > $OUT/steady.txt && cut -c1-150 $OUT/steady.txt | grep -E "steady|maxpool|apply_resbn|apply_kernel"
rm -rf $OUT/prof
