#!/bin/bash
# Phase stamps (clock read first) of the ConvNet step kernels, plain and forced, with starts.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4zb && mkdir -p $OUT
DPA_EXT_SO=$PWD/ddp_practice_amd/_C_timing.so timeout -k 10 120 python -u scripts/stamp_step.py --starts > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
DPA_EXT_SO=$PWD/ddp_practice_amd/_C_timing.so timeout -k 10 120 python -u scripts/stamp_step.py --forced > $OUT/stamps_forced.txt 2>&1 || { tail -20 $OUT/stamps_forced.txt; exit 1; }
grep -v amdgpu.ids $OUT/stamps.txt; grep -E "blocks=" $OUT/stamps_forced.txt
