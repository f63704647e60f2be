#!/bin/bash
# Exchange-site A/B (DPA_XSITE_MODE: 0 as before, 1 plain ticket load, 2 epoch words advanced
# after the exchange, 3 both) on the forced (W>1-shaped) ConvNet step: stamps + steady busy;
# short-run headline with graph upload; new DDP / graph GPU tests.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && R=$PWD && OUT=$PWD/gpurun_out/${1:-r5o} && mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_dist_gpu.py tests/test_xgmi_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for g in 16 20; do
    timeout -k 10 100 python bench.py --steps 20 --warmup 5 --steps-per-graph $g --no-baseline --extra-dtypes "" --no-steady > $OUT/short_${g}_$i.json 2> $OUT/short_${g}_$i.err || { tail -5 $OUT/short_${g}_$i.err; exit 1; }
    echo "short(20/5) spg $g run $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/short_${g}_$i.json | head -1)"
    DPA_NO_GRAPH_UPLOAD=1 timeout -k 10 100 python bench.py --steps 20 --warmup 5 --steps-per-graph $g --no-baseline --extra-dtypes "" --no-steady > $OUT/shortnu_${g}_$i.json 2> $OUT/shortnu_${g}_$i.err || { tail -5 $OUT/shortnu_${g}_$i.err; exit 1; }
    echo "short(20/5) spg $g no-upload run $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/shortnu_${g}_$i.json | head -1)"
  done
done
for m in 0 1 2 3; do
  DPA_XSITE_MODE=$m DPA_EXT_SO=ddp_practice_amd/_C_timing.so timeout -k 10 200 python scripts/stamp_step.py --forced > $OUT/stamps_forced_m$m.txt 2>&1 || { tail -5 $OUT/stamps_forced_m$m.txt; exit 1; }
  echo "== mode $m"; grep -E "^(conv2_fwd|head_step|conv2_bwd|wgrad1|amp_sgd)" $OUT/stamps_forced_m$m.txt | cut -c1-260
done
for r in 1 2; do
  for m in 0 3 2 1; do
    DPA_XSITE_MODE=$m timeout -k 10 200 python bench.py --force-collectives --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 > $OUT/forced_m${m}_$r.json 2> $OUT/forced_m${m}_$r.err || { tail -5 $OUT/forced_m${m}_$r.err; exit 1; }
    echo "forced mode $m run $r $(grep -o '"ms_per_step": [0-9.]*\|"steady_ms": [0-9.]*' $OUT/forced_m${m}_$r.json | tr '\n' ' ')"
  done
done
