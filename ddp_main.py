"""Multi-GPU DDP + SyncBN + AMP ConvNet training launched with multiprocessing spawn.

Same CLI, environment contract, stdout and checkpoint as
/root/reference/ddp_main.py:
    python ddp_main.py --gpu 0,1 [-e 3] [-b 32]
``prepare()`` sets MASTER_ADDR=localhost, MASTER_PORT=19198 (override with the
``MASTER_PORT`` environment variable — the reference hard-codes it),
CUDA_VISIBLE_DEVICES=--gpu and WORLD_SIZE=#visible devices, then spawns one
process per GPU; each calls ``init_process_group("nccl", "env://")`` (RCCL over
xGMI underneath, native communicator), converts BatchNorm to SyncBatchNorm,
wraps the model in DistributedDataParallel (C++ reducer), trains with AMP
(autocast + GradScaler) on a DistributedSampler order, evaluates with a
reduce-to-rank-0 of (size, correct), and rank 0 saves ``ddp_checkpoint.pt`` =
``{"model": ddp.state_dict() ("module." keys), "scaler": scaler.state_dict()}``.

AMP dtype: --amp-dtype fp16 (reference default) | bf16 | fp32.
Without a GPU, --cpu-procs N runs the same program on N gloo CPU ranks.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def prepare():
    parser = argparse.ArgumentParser()
    parser.add_argument("--gpu", default="0,1")
    parser.add_argument("-e", "--epochs", default=3, type=int, metavar="N", help="number of total epochs to run")
    parser.add_argument("-b", "--batch_size", default=32, type=int, metavar="N", help="number of batchsize")
    parser.add_argument("--data-root", default="./data")
    parser.add_argument("--synthetic", action="store_true")
    parser.add_argument("--train-samples", type=int, default=None, help="synthetic train-set size (tests)")
    parser.add_argument("--test-samples", type=int, default=None, help="synthetic test-set size (tests)")
    parser.add_argument("--amp-dtype", default="fp16", choices=["fp16", "bf16", "fp32"])
    parser.add_argument("--no-graph", action="store_true")
    parser.add_argument("--no-sync-bn", action="store_true")
    parser.add_argument("--bucket-cap-mb", type=float, default=None)
    parser.add_argument("--cpu-procs", type=int, default=0, help="CPU/gloo ranks when no GPU is present")
    parser.add_argument("--checkpoint", default="ddp_checkpoint.pt")
    args = parser.parse_args()

    # The following environment variables are set to enable DDP
    os.environ["MASTER_ADDR"] = os.environ.get("DPA_MASTER_ADDR", "localhost")
    os.environ["MASTER_PORT"] = os.environ.get("MASTER_PORT", "19198")
    from ddp_practice_amd.runtime.device import select_devices

    select_devices(args.gpu)
    import torch

    world_size = torch.cuda.device_count()
    if world_size == 0:
        world_size = max(1, args.cpu_procs)
    os.environ["WORLD_SIZE"] = str(world_size)
    return args


def init_ddp(local_rank):
    import torch

    import ddp_practice_amd.distributed as dist

    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    os.environ["RANK"] = str(local_rank)
    os.environ["LOCAL_RANK"] = str(local_rank)
    dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo", init_method="env://")


def get_ddp_generator(seed=3407):
    import torch

    import ddp_practice_amd.distributed as dist

    local_rank = dist.get_rank()
    g = torch.Generator()
    g.manual_seed(seed + local_rank)
    return g


def main(local_rank, args):
    import torch

    import ddp_practice_amd.distributed as dist
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import MNIST, DeviceLoader, DistributedSampler
    from ddp_practice_amd.engine import TrainLoop, evaluate
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm

    init_ddp(local_rank)
    dev = torch.device("cuda", local_rank) if torch.cuda.is_available() else torch.device("cpu")
    amp = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": None}[args.amp_dtype]
    model = ConvNet(amp_dtype=amp).to(dev)  # autocast inside forward, as the reference
    if not args.no_sync_bn:
        model = convert_sync_batchnorm(model)
    model = DistributedDataParallel(model, device_ids=[local_rank] if dev.type == "cuda" else None,
                                    bucket_cap_mb=args.bucket_cap_mb)
    criterion = CrossEntropyLoss().to(dev)
    optimizer = SGD(model.parameters(), 1e-4)
    scaler = GradScaler(enabled=amp is not None) if amp is not None else None
    train_dataset = MNIST(root=args.data_root, train=True, force_synthetic=args.synthetic, n=args.train_samples)
    train_sampler = DistributedSampler(train_dataset)
    g = get_ddp_generator()
    act_dtype = amp if (amp is not None and dev.type == "cuda") else torch.float32
    train_dloader = DeviceLoader(train_dataset, batch_size=args.batch_size, shuffle=False, num_workers=4,
                                 pin_memory=True, sampler=train_sampler, generator=g, device=dev, dtype=act_dtype)
    test_dataset = MNIST(root=args.data_root, train=False, force_synthetic=args.synthetic, n=args.test_samples)
    test_sampler = DistributedSampler(test_dataset)
    test_dloader = DeviceLoader(test_dataset, batch_size=args.batch_size, shuffle=False, num_workers=2,
                                pin_memory=True, sampler=test_sampler, device=dev, dtype=act_dtype)
    loop = TrainLoop(model, criterion, optimizer, train_dloader, scaler, use_graph=not args.no_graph)
    for epoch in range(args.epochs):
        if local_rank == 0:
            print(f"begin training of epoch {epoch + 1}/{args.epochs}", flush=True)
        train_dloader.sampler.set_epoch(epoch)
        loop.run_epoch()
    if loop.graph_error is not None and local_rank == 0:
        print(f"[ddp_practice_amd] hipGraph capture failed, ran eagerly: {loop.graph_error!r}", file=sys.stderr)
    if local_rank == 0:
        print("begin testing", flush=True)
    correct, size = evaluate(model, test_dloader, comm=dist.default_comm(), dst=0)
    if local_rank == 0:
        acc = correct / size
        print(f"Accuracy is {acc:.2%}", flush=True)
    if local_rank == 0:
        state = {"model": model.state_dict()}
        if scaler is not None:
            state["scaler"] = scaler.state_dict()
        torch.save(state, args.checkpoint)
    dist.destroy_process_group()


if __name__ == "__main__":
    args = prepare()
    import torch.multiprocessing as mp

    time_start = time.time()
    mp.spawn(main, args=(args,), nprocs=int(os.environ["WORLD_SIZE"]))
    time_elapsed = time.time() - time_start
    print(f"\ntime elapsed: {time_elapsed:.2f} seconds")
