#!/bin/bash
# Lean exchange (experiment build _C_xslean.so: epoch words advanced after the peer reads, the
# clock read only when a poll waits): xGMI GPU tests on it, then the forced step A/B.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5x} && mkdir -p $OUT
DPA_EXT_SO=ddp_practice_amd/_C_xslean.so timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_xgmi_gpu.py tests/test_xgmi_ddp_gpu.py tests/test_dist_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in base lean; do
    E=""; [ $v = lean ] && E="DPA_EXT_SO=ddp_practice_amd/_C_xslean.so"
    env $E timeout -k 10 200 python bench.py --force-collectives --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/x_${v}_$i.json 2> $OUT/x_${v}_$i.err || { tail -5 $OUT/x_${v}_$i.err; exit 1; }
    echo "forced $v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/x_${v}_$i.json | head -1)"
  done
done
