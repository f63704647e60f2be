#!/bin/bash
# ResNet-50 (BASELINE config 5): GPU tests, native bench plain / forced-collective (the W>1
# step shape), PyTorch's own stack captured (torchref), steady kernel tables plain / forced.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4e && mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_resnet_gpu.py tests/test_conv_igemm_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_plain.json 2> $OUT/rn_plain.err || { tail -20 $OUT/rn_plain.err; exit 1; }
timeout -k 10 240 python -u bench.py --model resnet50 --force-collectives --steps 20 --warmup 5 > $OUT/rn_forced.json 2> $OUT/rn_forced.err || { tail -20 $OUT/rn_forced.err; exit 1; }
timeout -k 10 240 python -u bench.py --model resnet50 --resnet-impl torchref --steps 20 --warmup 5 > $OUT/rn_torchref.json 2> $OUT/rn_torchref.err || { tail -20 $OUT/rn_torchref.err; exit 1; }
for v in plain forced torchref; do echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_$v.json) $(grep -o '"hipgraph": [a-z]*' $OUT/rn_$v.json) $(grep -o '"capture_note": "[^"]*"' $OUT/rn_$v.json)"; done
cd /tmp
for v in plain forced; do
  F=""; [ $v = forced ] && F="--force-collectives"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$v -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 $F --steps 12 --warmup 3 > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { tail -5 $OUT/prof_$v.err; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof_$v -name "*kernel_trace.csv" | head -1) amp_sgd_large 5 > $OUT/steady_$v.txt && cut -c1-150 $OUT/steady_$v.txt | head -45
  rm -rf $OUT/prof_$v
done
