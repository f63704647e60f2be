#!/bin/bash
# Lane-group sums on DPP / permlane swaps instead of ds_bpermute chains (head GEMV, head BN2 sums, conv5x5 epilogue,
# wgrad bias sums); head 1024 vs 256 lanes A/B, plain / forced, stamps, steady tables.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4n && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_convnet_fused_gpu.py tests/test_xgmi_ddp_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B="--steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes"
for i in 1 2; do
  for nt in 256 1024; do
    DPA_HEAD_NT=$nt timeout -k 10 200 python -u bench.py $B "" > $OUT/p_${nt}_$i.json 2> $OUT/p_${nt}_$i.err || { tail -20 $OUT/p_${nt}_$i.err; exit 1; }
    DPA_HEAD_NT=$nt timeout -k 10 200 python -u bench.py --force-collectives $B "" > $OUT/f_${nt}_$i.json 2> $OUT/f_${nt}_$i.err || { tail -20 $OUT/f_${nt}_$i.err; exit 1; }
    echo "run $i nt $nt plain $(grep -o '"ms_per_step": [0-9.]*' $OUT/p_${nt}_$i.json) forced $(grep -o '"ms_per_step": [0-9.]*' $OUT/f_${nt}_$i.json)"
  done
done
DPA_EXT_SO=$PWD/ddp_practice_amd/_C_timing.so timeout -k 10 120 python -u scripts/stamp_step.py > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/stamps.txt
DPA_EXT_SO=$PWD/ddp_practice_amd/_C_timing.so timeout -k 10 120 python -u scripts/stamp_step.py --forced > $OUT/stamps_forced.txt 2>&1 || { tail -20 $OUT/stamps_forced.txt; exit 1; }
grep -v amdgpu.ids $OUT/stamps_forced.txt
cd /tmp
for v in plain forced; do
  F=""; [ $v = forced ] && F="--force-collectives"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$v -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py $F --steps 640 --warmup 64 --extra-dtypes "" --no-baseline --epochs 0 --no-steady > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { tail -20 $OUT/prof_$v.err; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/trace_steady.py $(find $OUT/prof_$v -name "*kernel_trace.csv" | head -1) amp_s 128 > $OUT/steady_$v.txt && cut -c1-140 $OUT/steady_$v.txt
  rm -rf $OUT/prof_$v
done
