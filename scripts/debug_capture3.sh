cd $GRAFT_REPO_ROOT
for st in flatcopy async_main hook_fenced hook_async hook_flatcopy reducer; do
  timeout -k 10 120 python scripts/debug_capture3.py $st > gpurun_out/cap3_$st.log 2>&1
  echo "$st rc=$?"; grep -E " ok|rror" gpurun_out/cap3_$st.log | tail -2
done
