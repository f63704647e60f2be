cd $GRAFT_REPO_ROOT
for st in sync_fwd sync_bwd ddp_bwd ddp_sync_fwd ddp_sync_bwd; do
  timeout -k 10 120 python scripts/debug_capture.py $st > gpurun_out/cap_$st.log 2>&1
  echo "$st rc=$?"; grep -E "ok|Error|error" gpurun_out/cap_$st.log | tail -3
done
