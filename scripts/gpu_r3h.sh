#!/bin/bash
# xGMI self-test fix: distributed GPU tests, the forced-collective step with the engine on
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/r3h
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py tests/test_xgmi_gpu.py tests/test_xgmi_ddp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3h/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --force-collectives --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > gpurun_out/r3h/forced.json 2> gpurun_out/r3h/forced.err || exit $?
DPA_FUSED_SYNC=0 DPA_FUSED_GRAD=0 timeout -k 10 200 python -u bench.py --force-collectives --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > gpurun_out/r3h/forced_unfused.json 2> gpurun_out/r3h/forced_unfused.err || exit $?
timeout -k 10 200 python -u bench.py --force-collectives --comm rccl --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > gpurun_out/r3h/forced_rccl.json 2> gpurun_out/r3h/forced_rccl.err || exit $?
