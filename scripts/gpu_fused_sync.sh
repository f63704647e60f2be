# Fused SyncBN exchange (csrc/comm/xsite.h): distributed GPU tests, then A/B benches
# (forced collectives at W=1 and 2 ranks sharing the GPU, fused vs DPA_FUSED_SYNC=0) + kernel profile
set -o pipefail
TAG=${1:-fs}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xgmi_ddp_gpu.py tests/test_xgmi_gpu.py tests/test_dist_gpu.py tests/test_convnet_fused_gpu.py > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
timeout -k 10 200 python bench.py --steps 2000 --warmup 64 > $OUT/plain.json 2> $OUT/plain.err || { tail $OUT/plain.err; exit 1; }
timeout -k 10 200 python bench.py --steps 2000 --warmup 64 --force-collectives > $OUT/forced.json 2> $OUT/forced.err || { tail $OUT/forced.err; exit 1; }
DPA_FUSED_SYNC=0 DPA_FUSED_GRAD=0 timeout -k 10 200 python bench.py --steps 2000 --warmup 64 --force-collectives > $OUT/forced_nofuse.json 2> $OUT/forced_nofuse.err || { tail $OUT/forced_nofuse.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 1000 --warmup 64 --share-gpu > $OUT/share2.json 2> $OUT/share2.err || { tail -30 $OUT/share2.err; exit 1; }
DPA_FUSED_SYNC=0 DPA_FUSED_GRAD=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 2 --steps 1000 --warmup 64 --share-gpu > $OUT/share2_nofuse.json 2> $OUT/share2_nofuse.err || { tail -30 $OUT/share2_nofuse.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $OUT/*.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 320 --warmup 32 --force-collectives > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
