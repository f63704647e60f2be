#!/bin/bash
# usage: bash scripts/ab_bench.sh OUT ROUNDS "BENCH ARGS" LABEL=SO [LABEL=SO ...]
#   SO: "default" (the in-tree _C.so), a path to an experiment build, or env:VAR=VAL (the default
#   build with that environment variable set)
# Same-box A/B of extension builds (ddp_practice_amd/build.py DPA_BUILD_TAG): bench.py with
# BENCH ARGS under each build (SO "default": the in-tree _C.so), interleaved ROUNDS times;
# one line per run with ms_per_step, appended to OUT.
#   e.g. bash scripts/ab_bench.sh gpurun_out/x/ab.txt 3 "--force-collectives --steps 2000 --warmup 50 \
#        --no-baseline --epochs 0" new=default old=ddp_practice_amd/_C_fullbar.so
set -o pipefail
OUT=$1; ROUNDS=$2; ARGS=$3; shift 3
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p "$(dirname "$OUT")"
echo "# bench.py $ARGS" >> "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    label=${spec%%=*}; so=${spec#*=}
    envs=()
    if [ "$so" = "default" ]; then unset DPA_EXT_SO
    elif [ "${so#env:}" != "$so" ]; then unset DPA_EXT_SO; envs=("${so#env:}")  # label=env:VAR=VAL
    else export DPA_EXT_SO=$so; fi
    line=$(env "${envs[@]}" timeout -k 10 300 python bench.py $ARGS 2> "$OUT.$label.err") || { echo "$label failed" >> "$OUT"; tail -20 "$OUT.$label.err"; exit 1; }
    ev=$(grep -m1 '^\[bench\] [0-9]* steps: wall' "$OUT.$label.err" || true)  # DPA_BENCH_EVENTS=1 runs
    echo "$label $r $(echo "$line" | grep -o '"ms_per_step": [0-9.]*' | head -1) $ev" >> "$OUT"
  done
done
unset DPA_EXT_SO
cat "$OUT"
