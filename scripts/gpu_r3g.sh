#!/bin/bash
# round-3 records: driver-style bench, the forced-collective (W>1-shaped) step on one GPU,
# shared-GPU supervisor rehearsals (2 and 4 ranks), ResNet-50 with the current defaults
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/r3g
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3g/bench_driver.json 2> gpurun_out/r3g/bench_driver.err || exit $?
timeout -k 10 200 python -u bench.py --force-collectives --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > gpurun_out/r3g/forced.json 2> gpurun_out/r3g/forced.err || exit $?
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 50 --epochs 0 --no-baseline --extra-dtypes "" > gpurun_out/r3g/plain.json 2> gpurun_out/r3g/plain.err || exit $?
timeout -k 10 300 python -u bench.py --gpus 2 --share-gpu --steps 200 --warmup 20 --epochs 1 > gpurun_out/r3g/share2.json 2> gpurun_out/r3g/share2.err || exit $?
timeout -k 10 300 python -u bench.py --gpus 4 --share-gpu --steps 200 --warmup 20 --epochs 1 > gpurun_out/r3g/share4.json 2> gpurun_out/r3g/share4.err || exit $?
timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r3g/resnet.json 2> gpurun_out/r3g/resnet.err || exit $?
