set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x > gpurun_out/t2.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/t2.log
timeout -k 10 300 python bench.py --steps 2000 --warmup 64 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; echo "bench rc=$?"; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-graph > gpurun_out/bench1_nograph.json 2> gpurun_out/bench1_nograph.err; echo "bench nograph rc=$?"; cat gpurun_out/bench1_nograph.json; tail -5 gpurun_out/bench1_nograph.err
