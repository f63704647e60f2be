#!/bin/bash
# Pre-checked AMP step at W>1 (fused DDP over xGMI, NaN-poison agreement): full GPU tier,
# forced-collective A/B (DPA_PRECHECK=0), plain bench.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && R=$PWD && OUT=$PWD/gpurun_out/${1:-r5r} && mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new old; do
    E=""; [ $v = old ] && E="DPA_PRECHECK=0"
    env $E timeout -k 10 200 python bench.py --force-collectives --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/f_${v}_$i.json 2> $OUT/f_${v}_$i.err || { tail -5 $OUT/f_${v}_$i.err; exit 1; }
    echo "forced $v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/f_${v}_$i.json | head -1)"
    env $E timeout -k 10 200 python bench.py --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/p_${v}_$i.json 2> $OUT/p_${v}_$i.err || { tail -5 $OUT/p_${v}_$i.err; exit 1; }
    echo "plain $v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/p_${v}_$i.json | head -1)"
  done
done
for i in 1 2; do
  for v in atomic plain; do
    E=""; [ $v = plain ] && E="DPA_EXT_SO=ddp_practice_amd/_C_xsplain.so"
    env $E timeout -k 10 200 python bench.py --force-collectives --steps 2000 --warmup 50 --no-baseline --extra-dtypes "" --epochs 0 --no-steady > $OUT/x_${v}_$i.json 2> $OUT/x_${v}_$i.err || { tail -5 $OUT/x_${v}_$i.err; exit 1; }
    echo "forced epoch-advance $v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/x_${v}_$i.json | head -1)"
  done
done
for i in 1 2 3; do
  for v in first last; do
    E=""; [ $v = last ] && E="DPA_BENCH_REMAINDER_LAST=1"
    env $E timeout -k 10 100 python bench.py --steps 20 --warmup 5 --no-baseline --extra-dtypes "" --no-steady > $OUT/s_${v}_$i.json 2> $OUT/s_${v}_$i.err || { tail -5 $OUT/s_${v}_$i.err; exit 1; }
    echo "short(20/5) remainder-$v $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/s_${v}_$i.json | head -1)"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $R/bench.py --force-collectives --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python3 $R/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) sgd 128 > $OUT/steady_forced.txt && cut -c1-150 $OUT/steady_forced.txt
rm -rf $OUT/prof
