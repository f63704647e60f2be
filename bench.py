#!/usr/bin/env python3
"""Flagship benchmark: ConvNet DDP + AMP training, images/s for the whole node
plus a measured 3-epoch wall clock.

Config (BASELINE.json): the reference's ddp_main.py training step — ConvNet
(29,034 params), batch 32 per rank (weak scaling), SGD(lr=1e-4), SyncBN,
AMP autocast + GradScaler (bf16 here), DistributedSampler order, synthetic
1x28x28 MNIST-shaped data, random-init weights.  One process per GPU over
RCCL (+ the xGMI engine).  Each timed step = data gather + forward + loss +
backward (+ SyncBN / DDP all-reduces) + unscale/inf-check + SGD + scale
update, replayed from captured hipGraphs.

    python bench.py [--gpus N] [--steps K] [--warmup W]
        N > 1 without WORLD_SIZE in the environment: this process launches the N
        ranks itself (one per GPU, like the reference's mp.spawn,
        /root/reference/ddp_main.py:173-178) before touching the GPU.
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
        N ranks started by torchrun (RANK / LOCAL_RANK / WORLD_SIZE from the env).

What one run measures (rank 0 prints ONE JSON line):
  1. the reference's whole program on this node: 3 epochs over the 60k-sample
     train set (DistributedSampler shards, graph-replayed full batches + the
     eager tail batch) and the sharded test pass -> ``wall_3epoch_s``,
     ``epoch_img_s``, ``accuracy``; ``process_wall_3epoch_s`` adds process
     start-up (interpreter, imports, rendezvous) as the reference's timer does;
  2. the headline: exactly ``--warmup`` untimed then exactly ``--steps`` timed
     training steps, barrier + synchronize on both sides, max over ranks;
  3. the same-node baseline: the reference's step on PyTorch's own modules,
     autocast, GradScaler, SGD, SyncBatchNorm and DDP
     (ddp_practice_amd/utils/reference_step.py), same dtype -> ``vs_baseline``
     = value / baseline.  The reference's published number (other hardware,
     fp32, end to end) stays a labelled ``published_ref_img_s``.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) + 3-epoch wall-clock, MNIST ConvNet at 1/2/4/8 MI355X"
# 180,000 train images / 22.72 s (origin_main.py, 1 GPU, fp32) and / 30.82 s (ddp_main.py, W=2)
PUBLISHED_IMG_S = {1: 7923.0, 2: 5840.0}
PUBLISHED_WALL_S = {1: 22.72, 2: 30.82}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--amp-dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--impl", default="native", choices=["native", "torch"],
                    help="native = this framework (headline); torch = the reference step on torch's stack")
    ap.add_argument("--steps-per-graph", type=int, default=16)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-sync-bn", action="store_true")
    ap.add_argument("--epochs", type=int, default=3, help="epochs of the measured wall-clock run (0: skip)")
    ap.add_argument("--no-baseline", action="store_true", help="skip the same-node torch baseline")
    ap.add_argument("--baseline-steps", type=int, default=200)
    ap.add_argument("--force-collectives", action="store_true",
                    help="profiling: run the DDP/SyncBN collective path even at --gpus 1")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: every rank on cuda:0, all-reduces on the xGMI engine (not the metric)")
    ap.add_argument("--comm", default=None, choices=["auto", "rccl", "xgmi"],
                    help="collective algorithm selection (auto: xGMI engine where it is faster, else RCCL)")
    ap.add_argument("--model", default="convnet", choices=["convnet", "resnet50"],
                    help="convnet = the headline config; resnet50 = BASELINE.json stress config 5")
    ap.add_argument("--resnet-impl", default="native", choices=["native", "torch"],
                    help="resnet50: native NHWC kernels, or the plain torch module path (comparison)")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--train-samples", type=int, default=60000, help="synthetic train-set size (tests only)")
    ap.add_argument("--test-samples", type=int, default=10000, help="synthetic test-set size (tests only)")
    ap.add_argument("--out", default=None, help="also append the JSON line to this file")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned(local_rank: int, argv: list[str], world: int, port: int, t0: float) -> None:
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      DPA_BENCH_T0=repr(t0))
    run_rank(parse(argv))


def launch(args, argv: list[str]) -> int:
    """``--gpus N`` with no launcher: start N ranks (before any GPU call in this process)."""
    import torch

    n = args.gpus
    visible = torch.cuda.device_count()  # does not initialise the HIP runtime on this image
    if visible == 0:
        print(f"bench.py: no GPU visible: {n} CPU ranks over gloo (plumbing only, not the metric)", file=sys.stderr)
    elif not args.share_gpu and n > visible:
        print(f"bench.py: --gpus {n} but only {visible} GPU(s) are visible "
              f"(use --share-gpu for a one-GPU rehearsal)", file=sys.stderr)
        return 2
    if args.share_gpu and visible < 1:
        print("bench.py: --share-gpu needs one visible GPU", file=sys.stderr)
        return 2
    import torch.multiprocessing as mp

    t0 = time.time()
    try:
        mp.spawn(_spawned, args=(argv, n, _free_port(), t0), nprocs=n, join=True)
    except Exception as e:  # noqa: BLE001 - a rank failed: report and exit non-zero
        print(f"bench.py: a rank failed: {e}", file=sys.stderr)
        return 1
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch(args, argv)
    if "WORLD_SIZE" in os.environ:
        import torch

        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; measuring {world} ranks", file=sys.stderr)
        ngpu = torch.cuda.device_count()
        if ngpu and not args.share_gpu and int(os.environ.get("LOCAL_WORLD_SIZE", world)) > ngpu:
            print(f"bench.py: {os.environ.get('LOCAL_WORLD_SIZE', world)} local ranks but "
                  f"{torch.cuda.device_count()} visible GPU(s)", file=sys.stderr)
            return 2
    run_rank(args)
    return 0


# ----------------------------------------------------------------------------- helpers
def _force_collectives():
    """Profiling/rehearsal: run the DDP + SyncBN collective code path in a world of one."""
    from ddp_practice_amd.parallel import comm as _comm

    _comm.Communicator.force_active = True
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")


def _process_t0() -> float:
    if "DPA_BENCH_T0" in os.environ:
        return float(os.environ["DPA_BENCH_T0"])
    try:
        import psutil

        return psutil.Process(os.getpid()).create_time()
    except Exception:  # noqa: BLE001
        return _IMPORT_T


_IMPORT_T = time.time()


def _comm_desc(c) -> str:
    name = type(c).__name__
    st = getattr(c, "xgmi_status", None)
    return f"{name} (xgmi {st})" if st else name


def _ranks_seen(c) -> int:
    import torch

    if c is None or c.world_size == 1:
        return 1
    t = torch.ones(1, dtype=torch.float32, device=c.device)
    c.all_reduce_(t, "sum")
    return int(round(float(t.item())))


def _emit(rec: dict, out: str | None) -> None:
    line = json.dumps(rec)
    print(line, flush=True)
    if out:
        with open(out, "a") as f:
            f.write(line + "\n")


class _Chunks:
    """Exactly ``n`` training steps as replays of a K-step graph plus one graph of the remainder,
    keeping the loader's device step counter inside the epoch's full batches."""

    def __init__(self, step, spg: int, loader, nfull: int, graphs: bool):
        from ddp_practice_amd.runtime import CapturedStep

        self.step, self.spg, self.loader, self.nfull = step, max(1, spg), loader, nfull
        self.graphs = graphs
        self._mk = lambda k: CapturedStep(step, warmup=1, steps_per_graph=k, enabled=graphs,
                                          pre_capture=lambda: loader.set_step(0))
        self.runners: dict = {}
        self.pos = 0
        self.capture_error = None

    def runner(self, k: int):
        r = self.runners.get(k)
        if r is None:
            r = self._mk(k)
            if self.graphs and not r.capture():
                self.capture_error = r.capture_error
            self.loader.set_step(0)
            self.pos = 0
            self.runners[k] = r
        return r

    def prepare(self, n: int) -> None:
        """Capture every graph ``run(n)`` needs (outside any timed region)."""
        if n >= self.spg:
            self.runner(self.spg)
        if n % self.spg:
            self.runner(n % self.spg)

    def _chunk(self, k: int) -> None:
        if self.pos + k > self.nfull:
            self.loader.set_step(0)
            self.pos = 0
        self.runners[k].run()
        self.pos += k

    def run(self, n: int) -> None:
        for _ in range(n // self.spg):
            self._chunk(self.spg)
        if n % self.spg:
            self._chunk(n % self.spg)


# ----------------------------------------------------------------------------- ConvNet
def run_rank(args) -> None:
    if args.model == "resnet50":
        return bench_resnet(args)
    import torch

    from ddp_practice_amd import distributed as ddist
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import DeviceLoader, DistributedSampler, synthetic
    from ddp_practice_amd.engine import TrainLoop, evaluate
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm

    if args.comm:
        os.environ["DPA_COMM"] = args.comm
    world = int(os.environ.get("WORLD_SIZE", "1"))
    gpu = torch.cuda.is_available()
    local_rank = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_gpu:
        os.environ["DPA_SHARED_GPU"] = "1"  # ranks share one device (ops/convnet_fused.py)
    if gpu:
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
    else:  # CPU plumbing (BASELINE config 1): torch modules, gloo, no graphs, fp32
        dev = torch.device("cpu")
        args.no_graph, args.no_baseline, args.amp_dtype = True, True, "fp32"

    def sync():
        if gpu:
            torch.cuda.synchronize()

    dist_path = world > 1 or args.force_collectives
    if args.force_collectives:
        _force_collectives()
    if dist_path:
        ddist.init_process_group(backend=("xgmi" if args.share_gpu else "nccl") if gpu else "gloo")
    comm = ddist.default_comm()
    rank = ddist.get_rank()
    amp = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[args.amp_dtype]
    B = args.batch_size

    train_ds = synthetic(args.train_samples, seed=1, name="synthetic-MNIST-train")
    test_ds = synthetic(args.test_samples, seed=2, name="synthetic-MNIST-test")

    def build(seed: int):
        torch.manual_seed(seed)
        model = ConvNet(amp_dtype=amp).to(dev)
        if dist_path:
            if not args.no_sync_bn:
                model = convert_sync_batchnorm(model)
            model = DistributedDataParallel(model, device_ids=[local_rank] if gpu else None)
        return model, SGD(model.parameters(), lr=1e-4), GradScaler(enabled=amp is not None)

    act = amp if amp is not None else torch.float32
    crit = CrossEntropyLoss().to(dev)
    rec_extra: dict = {}

    # 1. the reference's program: 3 epochs + sharded test, measured end to end
    if args.epochs > 0 and args.impl == "native":
        model, opt, scaler = build(0)
        g = torch.Generator()
        g.manual_seed(3407 + rank)
        tr = DeviceLoader(train_ds, batch_size=B, sampler=DistributedSampler(train_ds, num_replicas=world, rank=rank),
                          generator=g, device=dev, dtype=act)
        te = DeviceLoader(test_ds, batch_size=B, sampler=DistributedSampler(test_ds, num_replicas=world, rank=rank),
                          device=dev, dtype=act)
        loop = TrainLoop(model, crit, opt, tr, scaler if amp is not None else None,
                         use_graph=not args.no_graph, steps_per_graph=args.steps_per_graph)
        ddist.barrier()
        sync()
        t0 = time.perf_counter()
        for ep in range(args.epochs):
            tr.sampler.set_epoch(ep)
            loop.run_epoch()
        sync()
        t_train = time.perf_counter() - t0
        correct, size = evaluate(model, te, comm=comm if comm.active else None, dst=0)
        sync()
        ddist.barrier()
        t_all = time.perf_counter() - t0
        t_proc = time.time() - _process_t0()
        t_train, t_all, t_proc = (ddist.max_over_ranks(v) for v in (t_train, t_all, t_proc))
        imgs = args.epochs * len(train_ds)
        rec_extra.update({
            "wall_3epoch_s": round(t_all, 3),
            "process_wall_3epoch_s": round(t_proc, 3),
            "epoch_img_s": round(imgs / t_train, 1),
            "train_3epoch_s": round(t_train, 3),
            "epochs": args.epochs,
            "accuracy": round(correct / size, 4) if rank == 0 and size else None,
            "steps_per_rank_per_epoch": len(tr),
            "published_ref_wall_s": PUBLISHED_WALL_S.get(world),
        })
        if loop.graph_error is not None:
            rec_extra["graph_error_3epoch"] = repr(loop.graph_error)
        del loop, model, opt, scaler, tr, te

    # 2. the headline: exactly K timed steps after exactly W warm-up steps
    spg = 1 if args.no_graph else args.steps_per_graph
    if args.impl == "native":
        model, optimizer, scaler = build(1)
        fused_grad = dist_path and amp is not None and model.defer_grad_sync_to(optimizer)
        # no DDP: conv1's weight-gradient column sums run inside the fused AMP step (engine.TrainLoop does the same)
        slab_sink = not dist_path and amp is not None and model.set_slab_sink(optimizer)
        sampler = DistributedSampler(train_ds, num_replicas=world, rank=rank)
        loader = DeviceLoader(train_ds, batch_size=B, sampler=sampler, device=dev, dtype=act)
        images, labels = loader.static_batch()
        loader.start_epoch()
        nfull = len(sampler) // B
        from ddp_practice_amd.data import accepts_deferred

        defer = accepts_deferred(model, images)  # the gather runs inside conv1

        def step():
            loader.fill_(images, labels, defer=defer)
            out = model(images)
            loss = crit(out, labels)
            optimizer.zero_grad(set_to_none=True)
            if amp is not None:
                scaler.scale(loss).backward()
                scaler.step(optimizer)
                scaler.update()
            else:
                loss.backward()
                optimizer.step()

        chunks = _Chunks(step, spg, loader, nfull, graphs=not args.no_graph)
        chunks.prepare(args.warmup)
        chunks.prepare(args.steps)
        if chunks.capture_error is not None and rank == 0:
            print(f"[bench] graph capture failed, eager fallback: {chunks.capture_error!r}", file=sys.stderr)
        chunks.run(args.warmup)
        ddist.barrier()
        sync()
        t0 = time.perf_counter()
        chunks.run(args.steps)
        sync()
        ddist.barrier()
        dt = time.perf_counter() - t0
        captured = chunks.graphs and chunks.capture_error is None
        impl_desc = "native (fused HIP kernels, C++ reducer/communicator)" if gpu else \
            "CPU plumbing (torch modules, gloo; not the metric)"
        grad_avg = ("in AMP-SGD kernel (xGMI)" if fused_grad else "reducer all-reduce") if dist_path \
            else "none (1 rank)"
    else:
        from ddp_practice_amd.utils.reference_step import TorchReferenceStep

        ref = TorchReferenceStep(dev, amp, world, *train_ds.to_device(dev),
                                 DistributedSampler(train_ds, num_replicas=world, rank=rank).indices().to(dev), B,
                                 local_rank=local_rank, seed=1)
        dt = ref.time_steps(args.steps, args.warmup, ddist.barrier)
        captured, spg = False, 1
        impl_desc = "torch (nn modules, torch.autocast, torch GradScaler/SGD/SyncBatchNorm/DDP)"
        grad_avg = "torch DDP" if world > 1 else "none (1 rank)"
        del ref
    dt_max = ddist.max_over_ranks(dt)
    ms = dt_max / args.steps * 1e3
    img_s = B * world * args.steps / dt_max

    # 3. same-node baseline: the reference step on torch's own stack, same dtype
    base = None
    if args.impl == "native" and not args.no_baseline and not args.share_gpu:
        try:
            from ddp_practice_amd.utils.reference_step import TorchReferenceStep

            ref = TorchReferenceStep(dev, amp, world, *train_ds.to_device(dev),
                                     DistributedSampler(train_ds, num_replicas=world, rank=rank).indices().to(dev),
                                     B, local_rank=local_rank, seed=1)
            n_b = max(args.baseline_steps, 1)
            tb = ddist.max_over_ranks(ref.time_steps(n_b, 20, ddist.barrier))
            base = B * world * n_b / tb
            rec_extra["baseline_ms_per_step"] = round(tb / n_b * 1e3, 4)
            del ref
        except Exception as e:  # noqa: BLE001 - the baseline is context, never the metric
            rec_extra["baseline_error"] = f"{type(e).__name__}: {e}"
    elif args.share_gpu:
        rec_extra["baseline_error"] = "skipped: --share-gpu rehearsal"

    seen = _ranks_seen(comm if dist_path else None)
    if rank == 0:
        pub = PUBLISHED_IMG_S.get(world)
        rec = {
            "metric": METRIC,
            "value": round(img_s, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / base, 3) if base else None,
            "baseline": "same-node torch reference step (ddp_practice_amd/utils/reference_step.py), same dtype",
            "baseline_same_node_img_s": round(base, 1) if base else None,
            "published_ref_img_s": pub,
            "published_ref_note": "BASELINE.md: reference fp32/fp16 end-to-end run on unstated NVIDIA GPUs",
            "dtype": args.amp_dtype,
            "data": f"synthetic 1x28x28 MNIST-shaped uint8 ({len(train_ds)} train / {len(test_ds)} test), "
                    "random-init weights",
            "config": {
                "model": "ConvNet (2x[Conv5x5-BN-ReLU-MaxPool2] + Linear(1568,10), 29,034 params)",
                "global_batch": B * world,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "per_rank_batch": B,
                "impl": impl_desc,
                "sync_bn": dist_path and not args.no_sync_bn,
                "amp": f"autocast {args.amp_dtype} + GradScaler" if amp is not None else "fp32",
                "optimizer": "SGD(lr=1e-4)",
                "hipgraph": bool(captured),
                "steps_per_graph": spg,
                "comm": _comm_desc(comm) if dist_path else "none (1 rank)",
                "grad_avg": grad_avg,
                "shared_gpu": bool(args.share_gpu),
            },
            "ranks_seen": seen,
            "per_rank_max_s": round(dt_max, 6),
        }
        rec.update(rec_extra)
        _emit(rec, args.out)
    ddist.destroy_process_group()


# ----------------------------------------------------------------------------- ResNet-50
def bench_resnet(args):
    """ResNet-50 training step (BASELINE.json config 5): channels-last AMP + GradScaler,
    SyncBN + DDP over RCCL for N > 1, synthetic 3x224x224 batch, replayed from a hipGraph
    (--no-graph: eager).  Exactly --warmup untimed and --steps timed steps."""
    import torch

    from ddp_practice_amd import distributed as ddist
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.models import resnet50
    from ddp_practice_amd.ops.head import cross_entropy
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm
    from ddp_practice_amd.runtime import CapturedStep

    if args.comm:
        os.environ["DPA_COMM"] = args.comm
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_gpu:
        os.environ["DPA_SHARED_GPU"] = "1"  # ranks share one device (ops/convnet_fused.py)
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

    # the step is hundreds of launches: capture it (after warm-up, so any library
    # algorithm search is done) and replay, or host overhead becomes the bound
    runner = CapturedStep(step, warmup=2, steps_per_graph=1, enabled=not args.no_graph)
    captured = runner.capture() if not args.no_graph else False
    if not captured and not args.no_graph and rank == 0:
        print(f"[bench] graph capture failed, eager: {runner.capture_error!r}", file=sys.stderr)
    for _ in range(args.warmup):
        runner.run()
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
    c = ddist.default_comm()
    seen = _ranks_seen(c if dist_path else None)
    if rank == 0:
        _emit({
            "metric": "images/sec (whole node), ResNet-50 stress config (BASELINE.json config 5)",
            "value": round(img_s, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.amp_dtype,
            "data": f"synthetic 3x{args.image_size}x{args.image_size}, random-init weights",
            "config": {"model": "ResNet-50 (25,557,032 params)", "global_batch": bs * world, "seq_len": None,
                       "parallelism": f"dp{world}", "per_rank_batch": bs, "impl": args.resnet_impl,
                       "sync_bn": dist_path and not args.no_sync_bn, "optimizer": "SGD(lr=1e-4)",
                       "comm": _comm_desc(c) if dist_path else "none", "hipgraph": bool(captured),
                       "shared_gpu": bool(args.share_gpu)},
            "ranks_seen": seen, "per_rank_max_s": round(dt, 6),
        }, args.out)
    ddist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
