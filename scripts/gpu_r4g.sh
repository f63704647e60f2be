#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/r4g
timeout -k 10 200 python -u scripts/exp/dbg_ddp_graph.py > gpurun_out/r4g/dbg.txt 2>&1; cat gpurun_out/r4g/dbg.txt | grep -v amdgpu.ids
