# ResNet-50: kernel-trace stats of the native and torch paths (1 GPU, bs 128)
set -o pipefail
TAG=${1:-rnprof}; BS=${2:-128}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/native -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --batch-size $BS --steps 10 --warmup 3 > $OUT/native.json 2> $OUT/native.err || { tail -20 $OUT/native.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/torch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet50 --resnet-impl torch --batch-size $BS --steps 10 --warmup 3 > $OUT/torch.json 2> $OUT/torch.err || { tail -20 $OUT/torch.err; exit 1; }
find $OUT -name "*kernel_stats.csv"
