# ResNet-50 bench: hipGraph replay vs eager, native vs torch module path
set -o pipefail
TAG=${1:-rng}
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
for impl in native torch; do
  for g in "" "--no-graph"; do
    n=${impl}${g:+_eager}
    timeout -k 10 300 python bench.py --model resnet50 --resnet-impl $impl --steps 20 --warmup 5 $g > $OUT/$n.json 2> $OUT/$n.err || { tail -20 $OUT/$n.err; exit 1; }
    grep -h "capture failed" $OUT/$n.err | head -2
    cut -c1-330 $OUT/$n.json
  done
done
