#!/bin/bash
# Round-4 baseline: ConvNet steady tables plain vs forced-collective (W>1 step shape),
# ResNet-50 plain vs forced-collective bench + forced steady table.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4a && mkdir -p $OUT
cd /tmp
for v in plain forced; do
  F=""; [ $v = forced ] && F="--force-collectives"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$v -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py $F --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { tail -20 $OUT/prof_$v.err; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof_$v -name "*kernel_trace.csv" | head -1) amp_sgd 128 > $OUT/steady_$v.txt && cut -c1-140 $OUT/steady_$v.txt
  rm -rf $OUT/prof_$v
done
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > $OUT/plain.json 2> $OUT/plain.err || { tail -20 $OUT/plain.err; exit 1; }
timeout -k 10 200 python -u bench.py --force-collectives --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > $OUT/forced.json 2> $OUT/forced.err || { tail -20 $OUT/forced.err; exit 1; }
echo "convnet plain $(grep -o '"ms_per_step": [0-9.]*' $OUT/plain.json) forced $(grep -o '"ms_per_step": [0-9.]*' $OUT/forced.json)"
timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 --no-baseline > $OUT/rn_plain.json 2> $OUT/rn_plain.err || { tail -20 $OUT/rn_plain.err; exit 1; }
timeout -k 10 240 python -u bench.py --model resnet50 --force-collectives --steps 20 --warmup 5 --no-baseline > $OUT/rn_forced.json 2> $OUT/rn_forced.err || { tail -20 $OUT/rn_forced.err; exit 1; }
echo "resnet plain $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_plain.json) forced $(grep -o '"ms_per_step": [0-9.]*' $OUT/rn_forced.json)"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_rnf -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --force-collectives --steps 12 --warmup 3 --no-baseline > $OUT/prof_rnf.json 2> $OUT/prof_rnf.err || { tail -5 $OUT/prof_rnf.err; exit 1; }
python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof_rnf -name "*kernel_trace.csv" | head -1) amp_sgd_large 5 > $OUT/steady_rn_forced.txt && cut -c1-140 $OUT/steady_rn_forced.txt | head -40
rm -rf $OUT/prof_rnf
