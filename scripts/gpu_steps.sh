#!/bin/bash
# usage: bash scripts/gpu_steps.sh TAG STEP [STEP ...]
# Named GPU measurement steps (each under its own time limit, output under gpurun_out/TAG/,
# the first failing step ends the run).  Steps:
#   push_ab      xGMI granule-pair pushes: one 16-B store (kept) vs two 8-B system-scope atomic
#                stores (scripts/exp/push_ab.py, W = 2 and 8 sharing the GPU; needs the
#                _C_pushatomic.so experiment build: DPA_EXTRA_CFLAGS=-DDPA_PUSH_ATOMIC2)
#   xsord_ab     forced step: exchange with epoch words advanced last / static peer unroll vs the
#                previous exchange (_C_xsold.so)
#   fp32_ab      fp32 step: merged conv2 backward launch (dynamic LDS) vs the two launches
#   cumask       does HSA_CU_MASK / ROC_GLOBAL_CU_MASK confine a process's kernels? (GEMM rate)
#   xsbar_ab     forced (W>1-shaped) ConvNet step: LDS-only exchange barriers vs __syncthreads
#                (needs _C_fullbar.so), 3 interleaved rounds
#   stamps       phase stamps of the fused ConvNet kernels, plain and forced (needs _C_timing.so)
#   steady       ConvNet steady-state kernel table (rocprofv3 kernel trace), plain and forced
#                (STEADY_MODES="plain forced fp32" adds the fp32 step)
#   rn_steady    ResNet-50 steady-state kernel table
#   bench        the driver's bench command and the default 2000-step run
#   rn_bench     ResNet-50 bench (bs 128, bf16)
#   rehearse8    bench.py with 8 ranks sharing the GPU under torchrun (scripts/gpu_rehearse.sh)
#   cli8         the 8-rank shared-GPU CLI tests (tests/test_cli_gpu.py -k eight; DPA_GPU_W8=1)
#   w8tests      the world-8 xGMI engine tests (DPA_GPU_W8=1)
#   ddp8         the 8-rank DDP + SyncBN xGMI tests, streaming the workers' stall reports
#   branches     do captured hipGraph fork/join branches overlap? (scripts/exp/graph_branches.py)
#   xtests       the xGMI / distributed / SyncBN / fused-ConvNet GPU tests (world-8 DDP excluded)
#   fp32det      fp32 slab-sink / bitwise-determinism tests, default and fp32 split-2 builds
#   bn_nt_ab     ResNet-50 A/B of non-temporal BN stores / loads
#   spin_ab      driver command, spinning vs yielding host waits
#   fixup_ab     ResNet-50 in-launch split-K weight-gradient reduction (tests, then A/B)
#   xsnoop_ab    forced step with the exchanges compiled out vs as built, and the plain step
#   xsbis_ab     the forced step's exchange cost bisected (experiment builds)
#   xglds_ab     AMP gradient average with an LDS-only epoch broadcast (W=2 tests + forced A/B)
#   bnu_ab       ResNet-50, BN rows in flight per lane 2 / 4 / 8
#   rn_bw        ResNet-50 per-kernel HBM bytes (PMC) and achieved bandwidth
#   rn_rehearse8 ResNet-50 DDP with 8 ranks sharing the card (torchrun, bs 16 per rank)
#   lpdyn_ab     bf16 conv2 backward tiles in dynamic LDS (tests + A/B)
#   plan_ab      driver window: lead + remainder graphs vs geometric graph sizes
#   fp32diag     per-key fp32 slab-sink vs separate-launch training (scripts/exp/fp32_sink_diff.py)
#   rn_rehearse2 / rn_rehearse4 / rn_rehearse4s / rn_rehearse4q / rn_rehearse8q / rn_rehearse8e
#                ResNet-50 DDP under torchrun sharing the card: world 2, 4 (graphs / serialized eager /
#                4 queues), 8 (4 queues / eager)
#   lpdyn_ab2    the same A/B as lpdyn_ab, more rounds, plain and forced
#   dg4_ab       conv2 data gradient at 4 workgroups per image (experiment build _C_dg4.so)
#   fp32dg_ab    fp32 conv2 data gradient split 4 vs 2 (experiment build _C_dgf2.so)
#   defer_ab     conv1 weight gradient inside the optimizer launch (DPA_DEFER_WGRAD1=1) vs as built
#   rn_knobs     ResNet-50 conv tuning knobs re-swept (wgrad blocks / min pixels, 1x1 pixel tile, stats defer)
#   rtenv_ab     HIP runtime knobs (HIP_FORCE_DEV_KERNARG, DEBUG_CLR_GRAPH_PACKET_CAPTURE) on the driver command
#   smoke        __graft_entry__.smoke()
#   gputests     the whole GPU test tier (as the driver runs it: world-8 rehearsals opt-in)
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && OUT=$PWD/gpurun_out/$TAG && mkdir -p "$OUT"
PYT="python -u -m pytest -x -v --timeout-method thread"
step() {
  case $1 in
    push_ab)
      for W in 2 8; do
        timeout -k 10 120 python scripts/exp/push_ab.py $W kept >> "$OUT/push_ab.txt" 2>&1 &&
        DPA_EXT_SO=ddp_practice_amd/_C_pushatomic.so timeout -k 10 120 python scripts/exp/push_ab.py $W atomic2 \
          >> "$OUT/push_ab.txt" 2>&1 || return 1
      done ;;
    xsord_ab)
      DPA_ALLOW_STALE_EXT=1 bash scripts/ab_bench.sh "$OUT/xsord_ab.txt" 3 "--force-collectives --steps 2000 --warmup 50 \
--no-baseline --epochs 0 --no-steady --extra-dtypes ," new=default old=ddp_practice_amd/_C_xsold.so ;;
    fp32_ab)
      bash scripts/ab_bench.sh "$OUT/fp32_ab.txt" 3 "--amp-dtype fp32 --steps 2000 --warmup 50 --no-baseline --epochs 0 \
--no-steady --extra-dtypes ," merged=default split=env:DPA_FP32_MERGED_BWD=0 ;;
    split_ab)  # workgroups per image of the conv2 forward / data gradient (experiment builds)
      for dt in fp32 bf16; do
        bash scripts/ab_bench.sh "$OUT/split_ab_$dt.txt" 3 "--amp-dtype $dt --steps 2000 --warmup 50 --no-baseline \
--epochs 0 --no-steady --extra-dtypes ," base=default fwd4=ddp_practice_amd/_C_fwd4.so dg4=ddp_practice_amd/_C_dg4.so || return 1
      done ;;
    fp32det)  # fp32 slab-sink step + bitwise determinism, current build then the fp32 split-2 build
      local K="fp32_plain_fused or bitwise_deterministic" rc
      timeout -k 10 300 $PYT --timeout 120 -p no:cacheprovider tests/test_convnet_fused_gpu.py -k "$K" \
        > "$OUT/fp32det_default.txt" 2>&1; rc=$?; echo "default rc=$rc" >> "$OUT/fp32det.txt"
      [ $rc -le 1 ] || return 1  # 0 pass, 1 test failure; anything else (timeout, abort): stop
      DPA_EXT_SO=$PWD/ddp_practice_amd/_C_sp2.so timeout -k 10 300 $PYT --timeout 120 -p no:cacheprovider \
        tests/test_convnet_fused_gpu.py -k "$K" > "$OUT/fp32det_sp2.txt" 2>&1; rc=$?
      echo "sp2 rc=$rc" >> "$OUT/fp32det.txt"; [ $rc -le 1 ] ;;
    fp32diag)  # localise the fp32 split-4 slab-sink mismatch (scripts/exp/fp32_sink_diff.py)
      timeout -k 10 200 $PYT --timeout 120 -p no:cacheprovider tests/test_convnet_fused_gpu.py -k bitwise \
        > "$OUT/fp32diag_bitwise.txt" 2>&1; local rc=$?; echo "bitwise rc=$rc" >> "$OUT/fp32diag.txt"
      [ $rc -le 1 ] || return 1
      local IFS=,; local runs=(${FP32DIAG_ARGS:-1 0,3 0,3 3}); unset IFS  # comma-separated "eager graph" pairs
      for a in "${runs[@]}"; do
        timeout -k 10 200 python scripts/exp/fp32_sink_diff.py $a >> "$OUT/fp32diag.txt" 2>&1 || return 1
      done
      DPA_EXT_SO=$PWD/ddp_practice_amd/_C_sp2.so timeout -k 10 200 python scripts/exp/fp32_sink_diff.py 3 0 \
        >> "$OUT/fp32diag.txt" 2>&1 ;;
    fixup_ab)  # ResNet-50: split-K weight-gradient reduction inside the launch, by split bound
      timeout -k 10 300 $PYT --timeout 120 -p no:cacheprovider tests/test_conv_igemm_gpu.py -k "fixup or wgrad" \
        > "$OUT/fixup_tests.txt" 2>&1 &&
      bash scripts/ab_bench.sh "$OUT/fixup_ab.txt" 2 "--model resnet50 --steps 100 --warmup 10 --no-baseline" \
        off=default sp8=env:DPA_WGRAD_FIXUP_MAXSP=8 sp32=env:DPA_WGRAD_FIXUP_MAXSP=32 all=env:DPA_WGRAD_FIXUP_MAXSP=100000 ;;
    xsnoop_ab)  # the forced step with every exchange compiled out (world 1) vs as built, and the plain step
      bash scripts/ab_bench.sh "$OUT/xsnoop_ab.txt" 3 "--force-collectives --steps 2000 --warmup 50 --no-baseline \
--epochs 0 --no-steady --extra-dtypes ," forced=default noop=ddp_practice_amd/_C_xsnoop.so &&
      bash scripts/ab_bench.sh "$OUT/xsnoop_ab.txt" 3 "--steps 2000 --warmup 50 --no-baseline --epochs 0 --no-steady \
--extra-dtypes ," plain=default ;;
    xsbis_ab)  # the forced step's exchange cost, bisected: no ticket / advance / barriers / AMP average
      local so=ddp_practice_amd
      bash scripts/ab_bench.sh "$OUT/xsbis_ab.txt" 3 "--force-collectives --steps 2000 --warmup 50 --no-baseline \
--epochs 0 --no-steady --extra-dtypes ," forced=default notk=$so/_C_xsnotk.so noadv=$so/_C_xsnoadv.so \
        nobar=$so/_C_xsnobar.so noxg=$so/_C_xsnoxg.so noop=$so/_C_xsnoop.so ;;
    xglds_ab)  # AMP gradient average: LDS-only epoch broadcast (experiment build) -- W=2 tests, then the forced A/B
      DPA_EXT_SO=$PWD/ddp_practice_amd/_C_xglds.so timeout -k 10 400 $PYT --timeout 170 -p no:cacheprovider \
        tests/test_xgmi_ddp_gpu.py -k "not 8-" > "$OUT/xglds_tests.txt" 2>&1 &&
      bash scripts/ab_bench.sh "$OUT/xglds_ab.txt" 3 "--force-collectives --steps 2000 --warmup 50 --no-baseline \
--epochs 0 --no-steady --extra-dtypes ," forced=default xglds=ddp_practice_amd/_C_xglds.so ;;
    bnu_ab)  # ResNet-50: rows in flight per lane of the NHWC BatchNorm kernels (experiment builds)
      bash scripts/ab_bench.sh "$OUT/bnu_ab.txt" 2 "--model resnet50 --steps 100 --warmup 10 --no-baseline" u4=default \
        u2=ddp_practice_amd/_C_bnu2.so u8=ddp_practice_amd/_C_bnu8.so ;;
    rn_bw)  # ResNet-50 per-kernel HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, one pass each) and bandwidth
      local RB="bench.py --model resnet50 --steps 3 --warmup 2 --no-graph --no-baseline"
      timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/bw_f" -o run -- python3 $RB \
        > "$OUT/bw_f.json" 2> "$OUT/bw_f.err" &&
      timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/bw_w" -o run -- python3 $RB \
        > "$OUT/bw_w.json" 2> "$OUT/bw_w.err" &&
      timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/bw_t" -o run -- python3 $RB \
        > "$OUT/bw_t.json" 2> "$OUT/bw_t.err" &&
      python3 scripts/bw_table.py "$(find "$OUT/bw_f" -name '*counter_collection.csv' -print -quit)" \
        "$(find "$OUT/bw_w" -name '*counter_collection.csv' -print -quit)" \
        "$(find "$OUT/bw_t" -name '*kernel_trace.csv' -print -quit)" 45 > "$OUT/rn_bw.txt" &&
      rm -rf "$OUT/bw_f" "$OUT/bw_w" "$OUT/bw_t" ;;
    rn_rehearse8)  # ResNet-50 DDP at world 8 on one card (torchrun, --share-gpu: 1/8 of the CUs per rank, bs 16)
      PYTHONFAULTHANDLER=1 DPA_BENCH_WATCHDOG=90 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py --model resnet50 --gpus 8 --share-gpu \
        --no-fallback --batch-size 16 --steps 10 --warmup 3 --no-baseline > "$OUT/rn_share_w8.json" \
        2> "$OUT/rn_share_w8.err" ;;
    rn_rehearse2)  # the same at world 2, Python stacks on a fatal signal (PYTHONFAULTHANDLER)
      PYTHONFAULTHANDLER=1 DPA_BENCH_WATCHDOG=90 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py --model resnet50 \
        --gpus 2 --share-gpu --no-fallback --batch-size 16 --steps 10 --warmup 3 --no-baseline \
        > "$OUT/rn_share_w2.json" 2> "$OUT/rn_share_w2.err" ;;
    rn_rehearse4s)  # world 4 on one card, eager and kernel-serialized (AMD_SERIALIZE_KERNEL=3): a fault is then
      # reported at the launch that caused it
      AMD_SERIALIZE_KERNEL=3 PYTHONFAULTHANDLER=1 DPA_BENCH_WATCHDOG=120 timeout -k 10 900 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py \
        --model resnet50 --gpus 4 --share-gpu --no-fallback --batch-size 16 --steps 4 --warmup 2 --no-baseline --no-graph \
        > "$OUT/rn_share_w4s.json" 2> "$OUT/rn_share_w4s.err" ;;
    rn_rehearse4)  # world 4 on one card, graph-captured as the bench runs it
      PYTHONFAULTHANDLER=1 DPA_BENCH_WATCHDOG=120 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py --model resnet50 \
        --gpus 4 --share-gpu --no-fallback --batch-size 16 --steps 10 --warmup 3 --no-baseline \
        > "$OUT/rn_share_w4.json" 2> "$OUT/rn_share_w4.err" ;;
    rn_rehearse4q)  # world 4 on one card, graph-captured, 4 HIP queues per rank (the 1-queue default from 3 ranks off)
      DPA_SHARED_HW_QUEUES=4 PYTHONFAULTHANDLER=1 DPA_BENCH_WATCHDOG=120 timeout -k 10 900 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py \
        --model resnet50 --gpus 4 --share-gpu --no-fallback --batch-size 16 --steps 10 --warmup 3 --no-baseline \
        > "$OUT/rn_share_w4q.json" 2> "$OUT/rn_share_w4q.err" ;;
    rn_rehearse8q)  # world 8 on one card, graph-captured, 4 HIP queues per rank
      DPA_SHARED_HW_QUEUES=4 PYTHONFAULTHANDLER=1 DPA_BENCH_WATCHDOG=120 timeout -k 10 900 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py \
        --model resnet50 --gpus 8 --share-gpu --no-fallback --batch-size 16 --steps 10 --warmup 3 --no-baseline \
        > "$OUT/rn_share_w8q.json" 2> "$OUT/rn_share_w8q.err" ;;
    rn_rehearse8e)  # world 8 on one card, eager (no graph)
      PYTHONFAULTHANDLER=1 DPA_BENCH_WATCHDOG=120 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py --model resnet50 \
        --gpus 8 --share-gpu --no-fallback --batch-size 16 --steps 4 --warmup 2 --no-baseline --no-graph \
        > "$OUT/rn_share_w8e.json" 2> "$OUT/rn_share_w8e.err" ;;
    lpdyn_ab)  # bf16 conv2 backward with the roles' tiles in dynamic LDS (DPA_LP_DYN_BWD=1): tests, then A/B
      DPA_LP_DYN_BWD=1 timeout -k 10 300 $PYT --timeout 120 -p no:cacheprovider tests/test_convnet_fused_gpu.py \
        -k "fwd_bwd or bitwise or slab_sink or prechecked" > "$OUT/lpdyn_tests.txt" 2>&1 &&
      bash scripts/ab_bench.sh "$OUT/lpdyn_ab.txt" 3 "--steps 2000 --warmup 50 --no-baseline --epochs 0 --no-steady \
--extra-dtypes ," static=env:DPA_LP_DYN_BWD=0 dyn=default ;;
    lpdyn_ab2)  # the same A/B, more rounds, plain and forced (in-kernel exchange sites)
      bash scripts/ab_bench.sh "$OUT/lpdyn_ab2.txt" 5 "--steps 2000 --warmup 50 --no-baseline --epochs 0 --no-steady \
--extra-dtypes ," static=env:DPA_LP_DYN_BWD=0 dyn=default &&
      bash scripts/ab_bench.sh "$OUT/lpdyn_ab2.txt" 3 "--force-collectives --steps 2000 --warmup 50 --no-baseline \
--epochs 0 --no-steady --extra-dtypes ," static=env:DPA_LP_DYN_BWD=0 dyn=default ;;
    plan_ab)  # the driver's 20-step window: lead graph + remainder (default) vs geometric graph sizes 1, 2, 4, ...
      DPA_BENCH_EVENTS=1 bash scripts/ab_bench.sh "$OUT/plan_ab.txt" 4 "--steps 20 --warmup 5" lead=default \
        geo=env:DPA_BENCH_PLAN=geo ;;
    dg4_ab)  # conv2 data gradient at 4 workgroups per image with the dynamic-LDS backward (experiment build)
      timeout -k 10 300 env DPA_EXT_SO=$PWD/ddp_practice_amd/_C_dg4.so $PYT --timeout 120 -p no:cacheprovider \
        tests/test_convnet_fused_gpu.py -k "fwd_bwd or bitwise" > "$OUT/dg4_tests.txt" 2>&1 &&
      bash scripts/ab_bench.sh "$OUT/dg4_ab.txt" 4 "--steps 2000 --warmup 50 --no-baseline --epochs 0 --no-steady \
--extra-dtypes ," dg2=default dg4=ddp_practice_amd/_C_dg4.so ;;
    rtenv_ab)  # HIP runtime knobs on the driver's command: kernel arguments in device memory, graph packet capture
      bash scripts/ab_bench.sh "$OUT/rtenv_ab.txt" 3 "--steps 20 --warmup 5 --no-baseline --epochs 0 --extra-dtypes ," \
        base=default kd1=env:HIP_FORCE_DEV_KERNARG=1 kd0=env:HIP_FORCE_DEV_KERNARG=0 gpc0=env:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 ;;
    defer_ab)  # conv1 weight gradient deferred into the optimizer's launch (DPA_DEFER_WGRAD1=1) vs as built
      bash scripts/ab_bench.sh "$OUT/defer_ab.txt" 3 "--steps 2000 --warmup 50 --no-baseline --epochs 0 --no-steady \
--extra-dtypes ," base=default defer=env:DPA_DEFER_WGRAD1=1 ;;
    rn_knobs)  # ResNet-50: re-sweep of the conv tuning knobs on this tree
      bash scripts/ab_bench.sh "$OUT/rn_knobs.txt" 2 "--model resnet50 --steps 100 --warmup 10 --no-baseline" base=default \
        wb384=env:DPA_WGRAD_BLOCKS=384 wb768=env:DPA_WGRAD_BLOCKS=768 mp512=env:DPA_WGRAD_MINPIX=512 \
        mp2048=env:DPA_WGRAD_MINPIX=2048 bp128=env:DPA_G1X1_BP=128 nodefer=env:DPA_STAT_DEFER_MIN=-1 ;;
    rn_minpix)  # ResNet-50: weight-gradient split floor (pixels per split) 1024 / 512 / 384 / 256
      bash scripts/ab_bench.sh "$OUT/rn_minpix.txt" 3 "--model resnet50 --steps 100 --warmup 10 --no-baseline" \
        mp1024=env:DPA_WGRAD_MINPIX=1024 mp512=default mp384=env:DPA_WGRAD_MINPIX=384 mp256=env:DPA_WGRAD_MINPIX=256 ;;
    rn_knobs2)  # ResNet-50: 64-channel tiles for small grids, wide-tile modes
      bash scripts/ab_bench.sh "$OUT/rn_knobs2.txt" 2 "--model resnet50 --steps 100 --warmup 10 --no-baseline" base=default \
        b64_256=env:DPA_G1X1_BN64_BELOW=256 b64_512=env:DPA_G1X1_BN64_BELOW=512 b64_1024=env:DPA_G1X1_BN64_BELOW=1024 \
        wide0=env:DPA_WIDE=0 wide2=env:DPA_WIDE=2 ;;
    fp32dg_ab)  # fp32 conv2 data gradient at 4 workgroups per image (default) vs 2 (_C_dgf2.so)
      bash scripts/ab_bench.sh "$OUT/fp32dg_ab.txt" 4 "--amp-dtype fp32 --steps 2000 --warmup 50 --no-baseline --epochs 0 \
--no-steady --extra-dtypes ," dg4=default dg2=ddp_practice_amd/_C_dgf2.so ;;
    spin_ab)  # busy-polled host waits (runtime/device.spin_sync) on the driver's command
      bash scripts/ab_bench.sh "$OUT/spin_ab.txt" 4 "--steps 20 --warmup 5" spin=env:DPA_SPIN_SYNC=1 yield=default ;;
    bn_nt_ab)  # ResNet-50: streaming (non-temporal) BN activation stores / loads (experiment builds)
      bash scripts/ab_bench.sh "$OUT/bn_nt_ab.txt" 2 "--model resnet50 --steps 100 --warmup 10 --no-baseline" base=default \
        ntst=ddp_practice_amd/_C_ntst.so ntld=ddp_practice_amd/_C_ntld.so ;;
    cumask)
      for e in "X=0" "HSA_CU_MASK=0:0-31" "ROC_GLOBAL_CU_MASK=0xffffffff"; do
        env $e timeout -k 10 60 python scripts/exp/cu_mask_probe.py >> "$OUT/cumask.txt" 2>&1 || return 1
      done ;;
    xsbar_ab)
      bash scripts/ab_bench.sh "$OUT/xsbar_ab.txt" 3 "--force-collectives --steps 2000 --warmup 50 --no-baseline \
--epochs 0 --no-steady --extra-dtypes ," ldsbar=default fullbar=ddp_practice_amd/_C_fullbar.so ;;
    stamps)
      DPA_EXT_SO=ddp_practice_amd/_C_timing.so timeout -k 10 120 python scripts/stamp_step.py > "$OUT/stamps_plain.txt" 2>&1 &&
      DPA_EXT_SO=ddp_practice_amd/_C_timing.so timeout -k 10 120 python scripts/stamp_step.py --forced \
        > "$OUT/stamps_forced.txt" 2>&1 ;;
    steady)
      for m in ${STEADY_MODES:-plain forced}; do
        local F=""; [ $m = forced ] && F=--force-collectives; [ $m = fp32 ] && F="--amp-dtype fp32"
        timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_$m" -o run -- python3 bench.py \
          --steps 640 --warmup 64 --extra-dtypes , --no-baseline --epochs 0 --no-steady $F > "$OUT/prof_$m.json" \
          2> "$OUT/prof_$m.err" || return 1
        python3 scripts/trace_steady.py "$(find "$OUT/prof_$m" -name '*kernel_trace.csv' -print -quit)" sgd 128 \
          > "$OUT/steady_$m.txt" || return 1
        rm -rf "$OUT/prof_$m"
      done ;;
    rn_steady)
      timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_rn" -o run -- python3 bench.py \
        --model resnet50 --steps 20 --warmup 5 > "$OUT/rn_steady.json" 2> "$OUT/rn_steady.err" &&
      python3 scripts/trace_steady.py "$(find "$OUT/prof_rn" -name '*kernel_trace.csv' -print -quit)" amp_sgd 5 \
        > "$OUT/rn_steady.txt" && rm -rf "$OUT/prof_rn" ;;
    bench)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" &&
      timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    rn_bench)
      timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 > "$OUT/rn_bench.json" 2> "$OUT/rn_bench.err" ;;
    rehearse8)
      bash scripts/gpu_rehearse.sh 8 "$TAG/rehearse8" > "$OUT/rehearse8.txt" 2>&1 ;;
    cli8)
      DPA_GPU_W8=1 timeout -k 10 600 $PYT --timeout 200 tests/test_cli_gpu.py -k eight > "$OUT/cli8.txt" 2>&1 ;;
    w8tests)  # the world-8 xGMI engine tests (opt-in: DPA_GPU_W8=1)
      DPA_GPU_W8=1 timeout -k 10 900 $PYT --timeout 330 tests/test_xgmi_gpu.py -k "8" > "$OUT/w8tests.txt" 2>&1 ;;
    cli8q4)  # the same with 4 HIP hardware queues per rank (the CU masks keep ranks apart)
      DPA_GPU_W8=1 DPA_SHARED_HW_QUEUES=4 timeout -k 10 600 $PYT --timeout 200 tests/test_cli_gpu.py -k "eight and spawn" \
        > "$OUT/cli8q4.txt" 2>&1 ;;
    cli8ab)  # the short 8-rank CLI test with the previous exchange build, then the current one
      DPA_GPU_W8=1 DPA_EXT_SO=$PWD/ddp_practice_amd/_C_xsold.so DPA_ALLOW_STALE_EXT=1 timeout -k 10 300 $PYT --timeout 200 \
        tests/test_cli_gpu.py -k "eight and spawn" > "$OUT/cli8_xsold.txt" 2>&1
      echo "xsold rc=$?" >> "$OUT/cli8ab.txt"
      DPA_GPU_W8=1 timeout -k 10 300 $PYT --timeout 200 tests/test_cli_gpu.py -k "eight and spawn" > "$OUT/cli8_new.txt" 2>&1
      echo "new rc=$?" >> "$OUT/cli8ab.txt" ;;
    rehearse8q4)
      DPA_SHARED_HW_QUEUES=4 bash scripts/gpu_rehearse.sh 8 "$TAG/rehearse8q4" > "$OUT/rehearse8q4.txt" 2>&1 ;;
    ddp8)
      DPA_GPU_W8=1 DPA_TEST_PROGRESS=1 timeout -k 10 400 $PYT -s --timeout 170 tests/test_xgmi_ddp_gpu.py -k "8-" \
        > "$OUT/ddp8.txt" 2>&1 ;;
    branches)
      for e in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "GPU_MAX_HW_QUEUES=8"; do
        env $e timeout -k 10 60 python scripts/exp/graph_branches.py >> "$OUT/branches.txt" 2>&1 || return 1
      done ;;
    xtests)
      timeout -k 10 900 $PYT --timeout 200 -m gpu tests/test_xgmi_gpu.py tests/test_dist_gpu.py tests/test_syncbn_gpu.py \
        tests/test_xgmi_ddp_gpu.py tests/test_convnet_fused_gpu.py -k "not 8-" > "$OUT/xtests.txt" 2>&1 ;;
    smoke)
      timeout -k 10 200 python __graft_entry__.py > "$OUT/smoke.txt" 2>&1 ;;
    gputests)
      timeout -k 10 1100 $PYT --timeout 200 -m gpu tests > "$OUT/gputests.txt" 2>&1 ;;
    *) echo "unknown step $1"; return 2 ;;
  esac
}
for s in "$@"; do
  echo "[gpu_steps] $s start $(date +%T)" | tee -a "$OUT/steps.log"
  step "$s" || { echo "[gpu_steps] $s FAILED" | tee -a "$OUT/steps.log"; exit 1; }
  echo "[gpu_steps] $s ok $(date +%T)" | tee -a "$OUT/steps.log"
done
