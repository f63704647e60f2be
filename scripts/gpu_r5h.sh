#!/bin/bash
# ConvNet conv2 split A/B: 4 workgroups per image for the conv2 forward (+ data gradient)
# vs the default 2, experiment builds loaded with DPA_EXT_SO; GPU tests on the s4 build.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5h} && mkdir -p $OUT
S4=$PWD/ddp_practice_amd/_C_s4.so; S4F=$PWD/ddp_practice_amd/_C_s4f.so
DPA_EXT_SO=$S4 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_convnet_fused_gpu.py > $OUT/pytest_s4.log 2>&1
rc=$?; tail -3 $OUT/pytest_s4.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in def s4 s4f; do
    case $v in def) E="";; s4) E="DPA_EXT_SO=$S4";; s4f) E="DPA_EXT_SO=$S4F";; esac
    env $E timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" > $OUT/b_${v}_$i.json 2> $OUT/b_${v}_$i.err || { tail -5 $OUT/b_${v}_$i.err; exit 1; }
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_${v}_$i.json | head -1) $(grep -o '"steady_ms_per_step": [0-9.]*' $OUT/b_${v}_$i.json)"
  done
done
