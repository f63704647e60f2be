#!/bin/bash
# AMP-SGD speculative pre-barrier update (rollback on a non-finite step)
# vs the previous build: optimizer + ConvNet tests, plain / forced A/B alternating.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4zf && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_convnet_fused_gpu.py tests/test_xgmi_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B="--steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes"
for i in 1 2 3; do
  for v in base new; do
    E=""; [ $v != new ] && E="DPA_EXT_SO=$PWD/ddp_practice_amd/_C_$v.so DPA_ALLOW_STALE_EXT=1"
    env $E timeout -k 10 200 python -u bench.py $B "" > $OUT/p_${v}_$i.json 2> $OUT/p_${v}_$i.err || { tail -20 $OUT/p_${v}_$i.err; exit 1; }
    env $E timeout -k 10 200 python -u bench.py --force-collectives $B "" > $OUT/f_${v}_$i.json 2> $OUT/f_${v}_$i.err || { tail -20 $OUT/f_${v}_$i.err; exit 1; }
    echo "run $i $v plain $(grep -o '"ms_per_step": [0-9.]*' $OUT/p_${v}_$i.json) forced $(grep -o '"ms_per_step": [0-9.]*' $OUT/f_${v}_$i.json)"
  done
done
