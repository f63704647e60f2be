#!/bin/bash
# Workgroup start skew of the ConvNet step kernels (phase stamps, start offset by block index).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4u && mkdir -p $OUT
DPA_EXT_SO=$PWD/ddp_practice_amd/_C_timing.so timeout -k 10 120 python -u scripts/stamp_step.py --starts > $OUT/stamps.txt 2>&1 || { tail -20 $OUT/stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/stamps.txt
