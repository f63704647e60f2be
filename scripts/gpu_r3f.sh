#!/bin/bash
# A/B in one run: head granule protocol (_C.so) vs the ticket protocol (_C_ticket.so, DPA_EXT_SO)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/r3f
for i in 1 2; do
  for v in new ticket; do
    if [ $v = ticket ]; then export DPA_EXT_SO=ddp_practice_amd/_C_ticket.so; else unset DPA_EXT_SO; fi
    timeout -k 10 120 python -u bench.py --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > gpurun_out/r3f/bench_${v}_$i.json 2>/dev/null || exit $?
  done
done
unset DPA_EXT_SO
bash scripts/gpu_convnet_trace.sh r3f/trace_new > gpurun_out/r3f/table_new.txt 2>&1 || exit $?
DPA_EXT_SO=ddp_practice_amd/_C_ticket.so bash scripts/gpu_convnet_trace.sh r3f/trace_ticket > gpurun_out/r3f/table_ticket.txt 2>&1 || exit $?
