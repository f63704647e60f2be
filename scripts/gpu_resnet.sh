# ResNet-50 stress config on 1 GPU: native vs torch module path, + kernel profile of the native step
set -o pipefail
TAG=${1:-rn}; BS=${2:-128}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python bench.py --model resnet50 --batch-size $BS --steps 20 --warmup 5 > $OUT/native.json 2> $OUT/native.err || { tail -20 $OUT/native.err; exit 1; }
cat $OUT/native.json
timeout -k 10 300 python bench.py --model resnet50 --resnet-impl torch --batch-size $BS --steps 20 --warmup 5 > $OUT/torch.json 2> $OUT/torch.err || { tail -20 $OUT/torch.err; exit 1; }
cat $OUT/torch.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --batch-size $BS --steps 10 --warmup 3 > $OUT/prof.json 2> $OUT/prof.err
echo "prof rc=$?"
