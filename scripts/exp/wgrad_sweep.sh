#!/bin/bash
# wgrad split heuristic sweep: network wgrad total from conv_bench for a few settings
for cfg in ${CFGS:-"768 1024" "1024 1024" "1536 512" "1024 512"}; do
  set -- $cfg
  DPA_WGRAD_BLOCKS=$1 DPA_WGRAD_MINPIX=$2 timeout -k 10 200 python -u scripts/exp/conv_bench.py > gpurun_out/wg_$1_$2.txt 2>&1 || exit 1
  echo "blocks=$1 minpix=$2: $(tail -1 gpurun_out/wg_$1_$2.txt)"
done
