#!/bin/bash
# conv1 weight gradient deferred into the fused AMP launch (5 launches per step): tests, bench,
# stamps, steady tables plain / forced
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/r4f && mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_convnet_fused_gpu.py -k "deferred_wgrad1 or slab_sink" -v -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
grep -E "PASS|FAIL|assert|Error" $OUT/tests.log | head -30
