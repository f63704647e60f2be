#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4i && mkdir -p $OUT
DPA_EXT_SO=$PWD/ddp_practice_amd/_C_timing.so timeout -k 10 120 python -u scripts/stamp_step.py > $OUT/stamps.txt 2>&1; grep -v amdgpu.ids $OUT/stamps.txt
DPA_DEFER_WGRAD1=0 DPA_EXT_SO=$PWD/ddp_practice_amd/_C_timing.so timeout -k 10 120 python -u scripts/stamp_step.py > $OUT/stamps0.txt 2>&1; grep -v amdgpu.ids $OUT/stamps0.txt
