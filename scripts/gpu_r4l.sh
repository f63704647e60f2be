#!/bin/bash
# SyncBN inside the ResNet statistics finishers (wide xGMI site): wide-site + dist + ResNet GPU
# tests, ResNet-50 bench plain / forced-collective, steady kernel tables of both.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4l && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_xgmi_gpu.py tests/test_resnet_gpu.py tests/test_conv_igemm_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > $OUT/rn_plain.json 2> $OUT/rn_plain.err || { tail -20 $OUT/rn_plain.err; exit 1; }
timeout -k 10 240 python -u bench.py --model resnet50 --force-collectives --steps 20 --warmup 5 > $OUT/rn_forced.json 2> $OUT/rn_forced.err || { tail -20 $OUT/rn_forced.err; exit 1; }
DPA_FUSED_SYNC=0 timeout -k 10 240 python -u bench.py --model resnet50 --force-collectives --steps 20 --warmup 5 > $OUT/rn_forced_launch.json 2> $OUT/rn_forced_launch.err || { tail -20 $OUT/rn_forced_launch.err; exit 1; }
for v in plain forced forced_launch; do echo "$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_$v.json)"; done
cd /tmp
for v in plain forced; do
  F=""; [ $v = forced ] && F="--force-collectives"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$v -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 $F --steps 12 --warmup 3 > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { tail -5 $OUT/prof_$v.err; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof_$v -name "*kernel_trace.csv" | head -1) amp_sgd_large 5 > $OUT/steady_$v.txt && cut -c1-150 $OUT/steady_$v.txt | head -30
  rm -rf $OUT/prof_$v
done
