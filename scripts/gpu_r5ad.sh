#!/bin/bash
# conv2_bwd's two roles sharing one exchange site (bf16 merged launch): xGMI / DDP / dist GPU
# tests, then the forced (W>1-shaped) step A/B against the previous build (_C_base.so).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5ad} && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_xgmi_gpu.py tests/test_xgmi_ddp_gpu.py tests/test_dist_gpu.py tests/test_convnet_fused_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for v in shared base; do
    E=""; [ $v = base ] && E="DPA_EXT_SO=ddp_practice_amd/_C_base.so DPA_ALLOW_STALE_EXT=1"
    env $E timeout -k 10 200 python bench.py --force-collectives --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/x_${v}_$i.json 2> $OUT/x_${v}_$i.err || { tail -5 $OUT/x_${v}_$i.err; exit 1; }
    echo "forced $v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/x_${v}_$i.json | head -1)"
  done
done
