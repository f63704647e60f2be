cd $GRAFT_REPO_ROOT
DPA_REDUCER_JOIN_EACH=1 timeout -k 10 120 python scripts/debug_capture.py ddp_bwd > gpurun_out/cap_je.log 2>&1; echo "join_each rc=$?"; grep -E "ok|rror" gpurun_out/cap_je.log | tail -3
