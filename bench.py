#!/usr/bin/env python3
"""Flagship benchmark: ConvNet DDP + AMP training step, images/s for the whole node.

Config (BASELINE.json): the reference's ddp_main.py training step — ConvNet
(29,034 params), batch 32 per rank (weak scaling), SGD(lr=1e-4), SyncBN,
AMP autocast + GradScaler (bf16 here), DistributedSampler order, synthetic
1x28x28 MNIST-shaped data, random-init weights.  One process per GPU over
RCCL.  Each timed step = data gather + forward + loss + backward (+ SyncBN /
DDP all-reduces) + unscale/inf-check + SGD + scale update, replayed from a
captured hipGraph.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_IMG_S = {1: 7923.0, 2: 5840.0}  # BASELINE.md (derived from README.md:201 / :466)


def _comm_desc() -> str:
    from ddp_practice_amd.parallel import comm

    c = comm.default_comm()
    name = type(c).__name__
    st = getattr(c, "xgmi_status", None)
    return f"{name} (xgmi {st})" if st else name


def _force_collectives():
    """Profiling/rehearsal: run the DDP + SyncBN collective code path in a world of one."""
    from ddp_practice_amd.parallel import comm as _comm

    _comm.Communicator.force_active = True
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--amp-dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--steps-per-graph", type=int, default=16)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-sync-bn", action="store_true")
    ap.add_argument("--force-collectives", action="store_true",
                    help="profiling: run the DDP/SyncBN collective path even at --gpus 1")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: every rank on cuda:0, all-reduces on the xGMI engine (not the metric)")
    ap.add_argument("--model", default="convnet", choices=["convnet", "resnet50"],
                    help="convnet = the headline config; resnet50 = BASELINE.json stress config 5")
    ap.add_argument("--resnet-impl", default="native", choices=["native", "torch"],
                    help="resnet50: native NHWC kernels, or the plain torch module path (comparison)")
    ap.add_argument("--image-size", type=int, default=224)
    args = ap.parse_args(argv)
    if args.model == "resnet50":
        return bench_resnet(args)

    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import ddp_practice_amd as dpa
    from ddp_practice_amd import distributed as ddist
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import DeviceLoader, DistributedSampler, synthetic
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.ops.head import cross_entropy
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm
    from ddp_practice_amd.runtime import CapturedStep

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("for --gpus N>1 launch with torchrun --nproc-per-node N")
    local_rank = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist_path = world > 1 or args.force_collectives
    if args.force_collectives:
        _force_collectives()
    if dist_path:
        ddist.init_process_group(backend="xgmi" if args.share_gpu else "nccl")
    rank = ddist.get_rank()

    amp = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[args.amp_dtype]
    torch.manual_seed(0)
    model = ConvNet(amp_dtype=amp).to(dev)
    if dist_path:
        if not args.no_sync_bn:
            model = convert_sync_batchnorm(model)
        model = DistributedDataParallel(model, device_ids=[local_rank])
    optimizer = SGD(model.parameters(), lr=1e-4)
    scaler = GradScaler(enabled=amp is not None)
    # DDP gradient averaging inside the fused AMP-SGD kernel (xGMI engine only)
    fused_grad = dist_path and amp is not None and model.defer_grad_sync_to(optimizer)

    ds = synthetic(60000, seed=1)
    sampler = DistributedSampler(ds, num_replicas=world, rank=rank)
    loader = DeviceLoader(ds, batch_size=args.batch_size, sampler=sampler, device=dev,
                          dtype=amp if amp is not None else torch.float32)
    images, labels = loader.static_batch()
    loader.start_epoch()
    nfull = len(sampler) // args.batch_size

    def step():
        loader.fill_(images, labels)
        out = model(images)
        loss = cross_entropy(out, labels)
        optimizer.zero_grad(set_to_none=True)
        scaler.scale(loss).backward()
        scaler.step(optimizer)
        scaler.update()

    spg = 1 if args.no_graph else args.steps_per_graph
    runner = CapturedStep(step, warmup=3, steps_per_graph=spg, enabled=not args.no_graph,
                          pre_capture=lambda: loader.set_step(0))
    captured = runner.capture() if not args.no_graph else False
    if not args.no_graph and not captured and rank == 0:
        print(f"[bench] graph capture failed, eager fallback: {runner.capture_error!r}", file=sys.stderr)

    # keep the device step counter inside the epoch: restart the order when needed
    state = {"pos": 0}

    def run_chunk():
        if state["pos"] + spg > nfull:
            loader.set_step(0)
            state["pos"] = 0
        runner.run()
        state["pos"] += spg

    n_warm = max(1, args.warmup // spg)
    for _ in range(n_warm):
        run_chunk()
    n_iter = max(1, args.steps // spg)
    steps = n_iter * spg
    ddist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_iter):
        run_chunk()
    torch.cuda.synchronize()
    ddist.barrier()
    t1 = time.perf_counter()
    dt = t1 - t0
    dt_max = ddist.max_over_ranks(dt)
    ms = dt_max / steps * 1e3
    img_s = args.batch_size * world * steps / dt_max
    if rank == 0:
        base = BASELINE_IMG_S.get(world, BASELINE_IMG_S[1])
        print(json.dumps({
            "metric": "images/sec (whole node) + 3-epoch wall-clock, MNIST ConvNet at 1/2/4/8 MI355X",
            "value": round(img_s, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": n_warm * spg,
            "ms_per_step": round(ms, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / base, 3),
            "dtype": args.amp_dtype,
            "data": "synthetic 1x28x28 MNIST-shaped uint8 (60k), random-init weights",
            "config": {
                "model": "ConvNet (2x[Conv5x5-BN-ReLU-MaxPool2] + Linear(1568,10), 29,034 params)",
                "global_batch": args.batch_size * world,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "per_rank_batch": args.batch_size,
                "sync_bn": dist_path and not args.no_sync_bn,
                "amp": f"autocast {args.amp_dtype} + GradScaler",
                "optimizer": "SGD(lr=1e-4)",
                "hipgraph": bool(captured),
                "comm": _comm_desc(),
                "grad_avg": ("in AMP-SGD kernel (xGMI)" if fused_grad else "reducer all-reduce") if dist_path
                else "none (1 rank)",
                "shared_gpu": bool(args.share_gpu),
                "steps_per_graph": spg,
                "est_3epoch_train_s": round(3 * len(loader) * ms / 1e3, 3),
                "baseline_img_s": base,
            },
        }), flush=True)
    ddist.destroy_process_group()


def bench_resnet(args):
    """ResNet-50 training step (BASELINE.json config 5): channels-last AMP + GradScaler,
    SyncBN + DDP over RCCL for N > 1, synthetic 3x224x224 batch, replayed from a hipGraph
    (--no-graph: eager)."""
    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from ddp_practice_amd import distributed as ddist
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.models import resnet50
    from ddp_practice_amd.ops.head import cross_entropy
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist_path = world > 1 or args.force_collectives
    if args.force_collectives:
        _force_collectives()
    if dist_path:
        ddist.init_process_group(backend="xgmi" if args.share_gpu else "nccl")
    rank = ddist.get_rank()
    amp = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[args.amp_dtype]
    bs = args.batch_size if args.batch_size != 32 else 128
    torch.manual_seed(0)
    model = resnet50(amp_dtype=amp, fused=args.resnet_impl == "native").to(dev)
    if args.resnet_impl == "torch":
        model = model.to(memory_format=torch.channels_last)
    if dist_path:
        if not args.no_sync_bn:
            model = convert_sync_batchnorm(model)
        model = DistributedDataParallel(model, device_ids=[local_rank])
    optimizer = SGD(model.parameters(), lr=1e-4)
    scaler = GradScaler(enabled=amp is not None)
    g = torch.Generator(device="cpu").manual_seed(rank)
    images = torch.rand(bs, 3, args.image_size, args.image_size, generator=g).to(dev)
    labels = torch.randint(0, 1000, (bs,), generator=g).to(dev)
    if args.resnet_impl == "torch":
        images = images.contiguous(memory_format=torch.channels_last)

    def step():
        if args.resnet_impl == "torch" and amp is not None:
            with torch.autocast("cuda", dtype=amp):
                out = model(images)
        else:
            out = model(images)
        loss = cross_entropy(out, labels)
        optimizer.zero_grad(set_to_none=True)
        scaler.scale(loss).backward()
        scaler.step(optimizer)
        scaler.update()

    # the step is ~600 launches: capture it (after warm-up, so MIOpen's algorithm
    # search is done) and replay, or the host's per-op overhead becomes the bound
    from ddp_practice_amd.runtime import CapturedStep

    runner = CapturedStep(step, warmup=max(1, args.warmup), steps_per_graph=1, enabled=not args.no_graph)
    captured = runner.capture() if not args.no_graph else False
    if not captured:
        if not args.no_graph and rank == 0:
            print(f"[bench] graph capture failed, eager: {runner.capture_error!r}", file=sys.stderr)
        for _ in range(max(1, args.warmup)):
            step()
    ddist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner.run()
    torch.cuda.synchronize()
    ddist.barrier()
    dt = ddist.max_over_ranks(time.perf_counter() - t0)
    ms = dt / args.steps * 1e3
    img_s = bs * world * args.steps / dt
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node), ResNet-50 stress config (BASELINE.json config 5)",
            "value": round(img_s, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": max(1, args.warmup), "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.amp_dtype,
            "data": f"synthetic 3x{args.image_size}x{args.image_size}, random-init weights",
            "config": {"model": "ResNet-50 (25,557,032 params)", "global_batch": bs * world, "seq_len": None,
                       "parallelism": f"dp{world}", "per_rank_batch": bs, "impl": args.resnet_impl,
                       "sync_bn": dist_path and not args.no_sync_bn, "optimizer": "SGD(lr=1e-4)",
                       "comm": _comm_desc() if dist_path else "none", "hipgraph": bool(captured),
                       "shared_gpu": bool(args.share_gpu)},
        }), flush=True)
    ddist.destroy_process_group()


if __name__ == "__main__":
    main()
