#!/bin/bash
# merged conv1-wgrad + AMP launch with an 8-word grid barrier: tests, A/B vs the 6-launch step
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4h && mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_convnet_fused_gpu.py tests/test_dist_gpu.py tests/test_xgmi_ddp_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for d in 1 0; do
    DPA_DEFER_WGRAD1=$d timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > $OUT/p${d}_$i.json 2> $OUT/p${d}_$i.err || { tail -20 $OUT/p${d}_$i.err; exit 1; }
    DPA_DEFER_WGRAD1=$d timeout -k 10 200 python -u bench.py --force-collectives --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > $OUT/f${d}_$i.json 2> $OUT/f${d}_$i.err || { tail -20 $OUT/f${d}_$i.err; exit 1; }
    echo "run $i defer=$d plain $(grep -o '"ms_per_step": [0-9.]*' $OUT/p${d}_$i.json) forced $(grep -o '"ms_per_step": [0-9.]*' $OUT/f${d}_$i.json)"
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) amp_s 128 > $OUT/steady.txt && cut -c1-140 $OUT/steady.txt
rm -rf $OUT/prof
