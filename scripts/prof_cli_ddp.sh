# cProfile of the torchrun CLI at W=1 (env set by hand, no agent): where the one-time costs go
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pcli}
mkdir -p $OUT && cd $OUT
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29581
timeout -k 10 300 python -m cProfile -o $OUT/ddp.prof $GRAFT_REPO_ROOT/ddp_main_torchrun.py --gpu 0 --synthetic > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
tail -2 $OUT/run.log
python -c "import pstats; pstats.Stats('$OUT/ddp.prof').sort_stats('cumtime').print_stats(45)" > $OUT/top.txt
python -c "import pstats; pstats.Stats('$OUT/ddp.prof').sort_stats('tottime').print_stats(25)" > $OUT/tot.txt
