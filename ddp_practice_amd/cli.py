"""Shared body of the three entry points (origin_main.py, ddp_main.py,
ddp_main_torchrun.py).

The reference repeats the same ~50-line ``main`` in every script
(/root/reference/origin_main.py:84-113, ddp_main.py:115-170,
ddp_main_torchrun.py:101-158); here the scripts keep the reference's
``prepare()`` / launch / timer contract and call ``run()``.

Stdout contract (rank 0 only): ``begin training of epoch e/E``,
``begin testing``, ``Accuracy is xx.xx%`` (the scripts print ``time elapsed``).

Additive flags (all optional; defaults reproduce the reference):
  --synthetic / --data-root / --train-samples / --test-samples   data
  --amp-dtype {fp16,bf16,fp32}        precision (reference: fp32 origin, fp16 DDP)
  --no-graph                          run every step eagerly (no hipGraph replay)
  --no-sync-bn / --bucket-cap-mb / --first-bucket-mb   DDP knobs
  --comm {auto,rccl,xgmi}             collective algorithm selection (parallel/comm.py)
  --impl {native,torch}               torch = the same program on PyTorch's own modules,
                                      autocast, GradScaler, SGD, SyncBatchNorm and DDP
                                      (parity / same-node baseline runs)
  --seed N                            model-init seed
  --model {convnet,resnet50}          resnet50 = BASELINE.json config 5 (ResNet-50, torchvision
                                      layout) on a synthetic ImageNet-shaped set
                                      (--image-size, --num-classes; data/imagenet.py)
  --resume PATH [--start-epoch N]     load {"model"[, "scaler"]} before training
  --watchdog-timeout S                abort + exit when no progress for S seconds (default at
                                      world size > 1: 600, torch's ProcessGroupNCCL default; 0 = off)
  --profile                           roctx ranges (rocprofv3 --marker-trace)
  --metrics-file PATH                 per-epoch JSONL (img/s, scale, ...) on rank 0
  --checkpoint PATH                   output file name
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time


def add_run_args(parser, amp_default: str, checkpoint: str, distributed: bool) -> None:
    parser.add_argument("--data-root", default="./data")
    parser.add_argument("--synthetic", action="store_true", help="use the synthetic MNIST-shaped dataset")
    parser.add_argument("--train-samples", type=int, default=None, help="synthetic train-set size (tests)")
    parser.add_argument("--test-samples", type=int, default=None, help="synthetic test-set size (tests)")
    parser.add_argument("--amp-dtype", default=amp_default, choices=["fp16", "bf16", "fp32"])
    parser.add_argument("--no-graph", action="store_true", help="run the training step eagerly")
    parser.add_argument("--seed", type=int, default=None)
    parser.add_argument("--checkpoint", default=checkpoint)
    parser.add_argument("--resume", default=None, help="checkpoint to load before training")
    parser.add_argument("--start-epoch", type=int, default=0, help="first epoch index (sampler seed) when resuming")
    parser.add_argument("--watchdog-timeout", type=float, default=None,
                        help="seconds without progress before aborting (env DPA_WATCHDOG_TIMEOUT; default 600 "
                             "at world size > 1, off for one process; 0 = off)")
    parser.add_argument("--profile", action="store_true", help="emit roctx ranges for rocprofv3 --marker-trace")
    parser.add_argument("--metrics-file", default=None, help="per-epoch JSONL metrics (rank 0)")
    parser.add_argument("--impl", default="native", choices=["native", "torch"],
                        help="torch: run the same program on PyTorch's own stack (parity / baseline)")
    parser.add_argument("--model", default="convnet", choices=["convnet", "resnet50"],
                        help="resnet50: ResNet-50 on synthetic 3 x S x S images (BASELINE.json config 5)")
    parser.add_argument("--image-size", type=int, default=224, help="resnet50: synthetic image side")
    parser.add_argument("--num-classes", type=int, default=1000, help="resnet50: synthetic label count")
    if distributed:
        parser.add_argument("--no-sync-bn", action="store_true")
        parser.add_argument("--bucket-cap-mb", type=float, default=None)
        parser.add_argument("--first-bucket-mb", type=float, default=None)
        parser.add_argument("--comm", default=None, choices=["auto", "rccl", "xgmi"],
                            help="collective algorithm: auto (size-selected xGMI engine / RCCL), rccl, xgmi")
        parser.add_argument("--share-gpu", action="store_true",
                            help="one-GPU rehearsal of the multi-rank program: every rank on the first --gpu "
                                 "device (ddp_main.py: one rank per --gpu entry), all-reduces and the in-kernel "
                                 "exchanges on the xGMI engine's peer stores, host collectives on gloo")


def apply_env(args) -> None:
    """Flags that must reach every rank before ``init_process_group`` (spawned children inherit the env)."""
    if getattr(args, "comm", None):
        os.environ["DPA_COMM"] = args.comm
    if getattr(args, "share_gpu", False):
        # ranks sharing one device: 3+ ranks' spinning in-kernel exchanges are not co-resident
        # on one card, so those take one launch per collective (ops/convnet_fused.py), and
        # each rank process gets one hardware queue (runtime/device.shared_gpu_env)
        from .runtime.device import shared_gpu_env

        gpus = [g for g in str(getattr(args, "gpu", "") or "").split(",") if g.strip()]
        world = int(os.environ["WORLD_SIZE"]) if "WORLD_SIZE" in os.environ else (len(gpus) or None)
        shared_gpu_env(world)


def share_gpu_rank_env(args, local_rank: int) -> None:
    """The per-rank part of ``--share-gpu`` (runtime/device.shared_cu_mask: this rank's own
    range of compute units from 3 ranks).  Before the rank's first HIP call, which
    ``torch.cuda.is_available()`` is."""
    if getattr(args, "share_gpu", False):
        from .runtime.device import shared_cu_mask

        shared_cu_mask(int(os.environ.get("WORLD_SIZE", "1")), local_rank)


def rank_device_index(args, local_rank: int) -> int:
    """The device a rank runs on: its local rank, or device 0 for every rank with --share-gpu."""
    return 0 if getattr(args, "share_gpu", False) else local_rank


def dist_backend(args) -> str:
    """init_process_group backend of a GPU rank: RCCL, or -- ranks sharing one device, which
    RCCL refuses -- the xGMI engine's rehearsal backend (parallel/comm.py init_process_group)."""
    return "xgmi" if getattr(args, "share_gpu", False) else "nccl"


def load_checkpoint(path: str, model, scaler=None) -> None:
    """Load a reference-format checkpoint ({"model": sd[, "scaler": sd]}) without unpickling code.

    Accepts both key styles (``layer1.0.weight`` and DDP's ``module.layer1.0.weight``).
    """
    import torch

    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = ck["model"]
    if all(k.startswith("module.") for k in sd):
        sd = {k[len("module."):]: v for k, v in sd.items()}
    model.load_state_dict(sd)
    if scaler is not None and "scaler" in ck and ck["scaler"]:
        scaler.load_state_dict(ck["scaler"])


DEFAULT_WATCHDOG_S = 600.0  # torch/distributed/constants.py:21 default_pg_timeout (ProcessGroupNCCL)


def watchdog_timeout(args, world: int) -> float:
    """The watchdog timeout of a run: --watchdog-timeout, else DPA_WATCHDOG_TIMEOUT, else
    on by default at world size > 1 (the reference's ``init_process_group("nccl")`` arms
    ProcessGroupNCCL's 10-minute watchdog: /root/reference/ddp_main.py:73).  0 = off."""
    t = getattr(args, "watchdog_timeout", None)
    if t is None and "DPA_WATCHDOG_TIMEOUT" in os.environ:
        t = float(os.environ["DPA_WATCHDOG_TIMEOUT"])
    if t is None:
        t = DEFAULT_WATCHDOG_S if world > 1 else 0.0
    return float(t)


def check_health(comm, where: str) -> None:
    """Raise on every rank when any rank's communicator reported an asynchronous error
    (parallel/comm.agree_on_errors): training must not go on, and no checkpoint may be
    written, after updates an exchange failure skipped or corrupted."""
    if comm is None or not getattr(comm, "active", False):
        return
    from ddp_practice_amd.parallel.comm import agree_on_errors

    err = agree_on_errors(comm)
    if err:
        raise RuntimeError(f"[ddp_practice_amd] communicator error {where}: {err}")


class _Metrics:
    def __init__(self, path: str | None, rank: int, world: int, device):
        self.path = path if rank == 0 else None
        self.world = world
        self.device = device
        self.t0 = None

    def start(self):
        if self.path is None:
            return
        self._sync()
        self.t0 = time.perf_counter()

    def _sync(self):
        import torch

        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def epoch(self, epoch: int, images: int, steps: int, scaler=None):
        if self.path is None:
            return
        self._sync()
        dt = time.perf_counter() - self.t0
        rec = {"epoch": epoch, "steps_per_rank": steps, "images": images, "seconds": round(dt, 4),
               "images_per_s": round(images / dt, 1) if dt > 0 else None, "world_size": self.world}
        if scaler is not None and scaler.is_enabled():
            rec["loss_scale"] = scaler.get_scale()
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")
        self.t0 = time.perf_counter()


_T0 = time.perf_counter()


def phase(name: str) -> None:
    """``DPA_PHASES=1``: print the time since this module was imported at each run phase (stderr)."""
    if os.environ.get("DPA_PHASES") == "1":
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            torch.cuda.synchronize()  # the mark covers the GPU work queued before it
        print(f"[phase pid={os.getpid()}] {name} +{time.perf_counter() - _T0:.3f}s", file=sys.stderr, flush=True)


def run(args, distributed: bool, local_rank: int = 0, generator_seed: int | None = None) -> None:
    """Build model/data/optimizer, train ``args.epochs`` epochs, test, save (rank 0)."""
    phase("run")
    import torch

    import ddp_practice_amd.distributed as dist
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import MNIST, DeviceLoader, DistributedSampler
    from ddp_practice_amd.engine import TrainLoop, evaluate
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.utils import FaultInjector, Watchdog, set_tracing, trace_range

    phase("imports")
    # The datasets (IDX read or host synthetic generation, numpy: releases the GIL in its
    # bulk ops) are built on a side thread while this one brings up the HIP context, the
    # native extension and the model; joined before the loaders need them.  A synthetic
    # MNIST set on a HIP device is instead generated in HBM by one kernel, on this thread
    # once the device is current (data/mnist.py synthetic(device=)).
    ds_box: dict = {}

    resnet = getattr(args, "model", "convnet") == "resnet50"
    from ddp_practice_amd.data.mnist import idx_available

    on_device = (not resnet and torch.cuda.is_available()
                 and (args.synthetic or not idx_available(args.data_root)))

    def _build_datasets():
        if on_device:
            return
        try:
            if resnet:  # no ImageNet reader (no network): the synthetic set, small by default
                from ddp_practice_amd.data import synthetic_imagenet

                kw = dict(classes=args.num_classes, hw=args.image_size)
                ds_box["train"] = synthetic_imagenet(args.train_samples or 1280, seed=1,
                                                     name="synthetic-imagenet-train", **kw)
                ds_box["test"] = synthetic_imagenet(args.test_samples or 256, seed=2,
                                                    name="synthetic-imagenet-test", **kw)
                return
            ds_box["train"] = MNIST(root=args.data_root, train=True, force_synthetic=args.synthetic,
                                    n=args.train_samples)
            ds_box["test"] = MNIST(root=args.data_root, train=False, force_synthetic=args.synthetic,
                                   n=args.test_samples)
        except BaseException as e:  # re-raised on the main thread
            ds_box["error"] = e

    ds_thread = threading.Thread(target=_build_datasets, name="dpa-datasets", daemon=True)
    ds_thread.start()
    if args.profile:
        set_tracing(True)
    if args.seed is not None:
        torch.manual_seed(args.seed)
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", rank_device_index(args, local_rank) if distributed else 0) if gpu else torch.device("cpu")
    rank = dist.get_rank() if distributed else 0
    world = dist.get_world_size() if distributed else 1
    comm = dist.default_comm() if distributed else None
    amp = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": None}[args.amp_dtype]

    native = getattr(args, "impl", "native") == "native"
    # autocast inside forward, as the reference; fused=False: torch's own modules
    if resnet:
        from ddp_practice_amd.models import resnet50

        model = resnet50(num_classes=args.num_classes, amp_dtype=amp, fused=native).to(dev)
    else:
        model = ConvNet(amp_dtype=amp, fused=native).to(dev)
    if native:
        scaler = GradScaler(enabled=True) if amp is not None else None
    else:
        scaler = torch.amp.GradScaler(dev.type) if amp is not None else None
    if args.resume:
        load_checkpoint(args.resume, model, scaler)
    if distributed and native:
        from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm

        if not args.no_sync_bn:
            model = convert_sync_batchnorm(model)
        model = DistributedDataParallel(model, device_ids=[dev.index] if gpu else None,
                                        bucket_cap_mb=args.bucket_cap_mb, first_bucket_mb=args.first_bucket_mb,
                                        # zero-copy buckets: the fused optimizer step reads them
                                        gradient_as_bucket_view=True)
    elif distributed:
        if not args.no_sync_bn and gpu:  # torch's SyncBatchNorm has no CPU path
            model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
        kw = {} if args.bucket_cap_mb is None else {"bucket_cap_mb": args.bucket_cap_mb}
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index] if gpu else None, **kw)
    criterion = (CrossEntropyLoss() if native else torch.nn.CrossEntropyLoss()).to(dev)
    optimizer = SGD(model.parameters(), 1e-4) if native else torch.optim.SGD(model.parameters(), 1e-4)
    phase("model")

    act_dtype = amp if (amp is not None and gpu) else torch.float32
    ds_thread.join()
    if "error" in ds_box:
        raise ds_box["error"]
    if on_device:
        ds_box["train"] = MNIST(root=args.data_root, train=True, force_synthetic=True, n=args.train_samples,
                                device=dev)
        ds_box["test"] = MNIST(root=args.data_root, train=False, force_synthetic=True, n=args.test_samples,
                               device=dev)
    train_dataset, test_dataset = ds_box["train"], ds_box["test"]
    if distributed:
        g = torch.Generator()
        g.manual_seed(generator_seed if generator_seed is not None else 3407 + rank)
        train_dloader = DeviceLoader(train_dataset, batch_size=args.batch_size, shuffle=False, num_workers=4,
                                     pin_memory=True, sampler=DistributedSampler(train_dataset), generator=g,
                                     device=dev, dtype=act_dtype)
        test_dloader = DeviceLoader(test_dataset, batch_size=args.batch_size, shuffle=False, num_workers=2,
                                    pin_memory=True, sampler=DistributedSampler(test_dataset), device=dev,
                                    dtype=act_dtype)
    else:
        train_dloader = DeviceLoader(train_dataset, batch_size=args.batch_size, shuffle=True, device=dev,
                                     dtype=act_dtype, num_workers=4, pin_memory=True)
        test_dloader = DeviceLoader(test_dataset, batch_size=args.batch_size, shuffle=True, device=dev,
                                    dtype=act_dtype, num_workers=2, pin_memory=True)

    phase("data")
    timeout = watchdog_timeout(args, world)
    watchdog = Watchdog(comm, timeout=timeout, tag=f"rank{rank}") if timeout > 0 else None
    faults = FaultInjector(rank, comm=comm)
    # ResNet-50: hundreds of launches per step, one step per captured graph is enough
    loop = TrainLoop(model, criterion, optimizer, train_dloader, scaler, use_graph=native and not args.no_graph,
                     steps_per_graph=1 if resnet else 16, watchdog=watchdog, faults=faults)
    metrics = _Metrics(args.metrics_file, rank, world, dev)
    metrics.start()
    try:
        for epoch in range(args.start_epoch, args.start_epoch + args.epochs):
            if rank == 0:
                print(f"begin training of epoch {epoch - args.start_epoch + 1}/{args.epochs}", flush=True)
            if distributed:
                train_dloader.sampler.set_epoch(epoch)
            loop.run_epoch()
            check_health(comm, f"after epoch {epoch - args.start_epoch + 1}")
            metrics.epoch(epoch, len(train_dataset), len(train_dloader), scaler)
            phase(f"epoch {epoch}")
        if loop.graph_error is not None and rank == 0:
            print(f"[ddp_practice_amd] hipGraph capture failed, ran eagerly: {loop.graph_error!r}", file=sys.stderr)
        if rank == 0:
            print("begin testing", flush=True)
        with trace_range("evaluate"):
            correct, size = evaluate(model, test_dloader, comm=comm, dst=0, native=native)
        if watchdog is not None:
            watchdog.tick()
        phase("evaluate")
        check_health(comm, "before saving the checkpoint")
        if rank == 0:
            print(f"Accuracy is {correct / size:.2%}", flush=True)
            with trace_range("checkpoint"):
                state = {"model": model.state_dict()}
                if scaler is not None and distributed:
                    state["scaler"] = scaler.state_dict()
                torch.save(state, args.checkpoint)
        if distributed and os.environ.get("DPA_CHECKPOINT_EVERY_RANK") == "1":
            # debugging / tests: every rank's own parameters (DDP keeps them bitwise equal)
            torch.save({"model": model.state_dict()}, f"{args.checkpoint}.rank{rank}")
    finally:
        if watchdog is not None:
            watchdog.stop()
    phase("saved")
    if distributed:
        dist.destroy_process_group()
    phase("done")
