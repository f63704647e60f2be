set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 320 --warmup 32 > $GRAFT_REPO_ROOT/gpurun_out/prof1/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof1/bench.err
echo "rc=$?"
find $GRAFT_REPO_ROOT/gpurun_out/prof1 -name "*.csv" | head
