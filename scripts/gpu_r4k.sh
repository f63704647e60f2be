#!/bin/bash
# BN statistics loads issued ahead of the activation loads (head, conv2_fwd prologue, conv2_bwd / wgrad prologues):
# ConvNet + xGMI tests, bench plain / forced, stamps, steady tables.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4k && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_convnet_fused_gpu.py tests/test_xgmi_ddp_gpu.py tests/test_xgmi_gpu.py tests/test_dist_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > $OUT/plain_$i.json 2> $OUT/plain_$i.err || { tail -20 $OUT/plain_$i.err; exit 1; }
  timeout -k 10 200 python -u bench.py --force-collectives --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > $OUT/forced_$i.json 2> $OUT/forced_$i.err || { tail -20 $OUT/forced_$i.err; exit 1; }
  echo "run $i plain $(grep -o '"ms_per_step": [0-9.]*' $OUT/plain_$i.json) forced $(grep -o '"ms_per_step": [0-9.]*' $OUT/forced_$i.json)"
done
DPA_EXT_SO=$PWD/ddp_practice_amd/_C_timing.so timeout -k 10 120 python -u scripts/stamp_step.py > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
cd /tmp
for v in plain forced; do
  F=""; [ $v = forced ] && F="--force-collectives"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$v -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py $F --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { tail -20 $OUT/prof_$v.err; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof_$v -name "*kernel_trace.csv" | head -1) amp_sgd 128 > $OUT/steady_$v.txt && cut -c1-140 $OUT/steady_$v.txt
  rm -rf $OUT/prof_$v
done
