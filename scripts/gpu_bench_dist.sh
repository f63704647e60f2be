# 1-GPU benches: plain, forced collectives (RCCL+xGMI at W=1), 2 ranks sharing the GPU (xGMI), + kernel profile of the forced run
set -o pipefail
TAG=${1:-bd}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python bench.py --steps 2000 --warmup 64 > $OUT/plain.json 2> $OUT/plain.err || { tail $OUT/plain.err; exit 1; }
cat $OUT/plain.json
timeout -k 10 200 python bench.py --steps 2000 --warmup 64 --force-collectives > $OUT/forced.json 2> $OUT/forced.err || { tail $OUT/forced.err; exit 1; }
cat $OUT/forced.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 1000 --warmup 64 --share-gpu > $OUT/share2.json 2> $OUT/share2.err || { tail -30 $OUT/share2.err; exit 1; }
cat $OUT/share2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 320 --warmup 32 --force-collectives > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
