#!/bin/bash
# Last check of the committed tree: every GPU test and the smoke entry point.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/${1:-r5last} && mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
