"""DDP + SyncBN + AMP ConvNet training launched by torchrun.

Same CLI and behaviour as /root/reference/ddp_main_torchrun.py:
    torchrun --standalone --nproc_per_node=2 ddp_main_torchrun.py --gpu 0,1
The elastic agent provides RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT; ``init_process_group("nccl")`` uses env://.  ``--gpu`` sets
CUDA_VISIBLE_DEVICES as in the reference (whose default "2,3" needs a 4+ GPU
node — pass ``--gpu 0,...,N-1`` for N ranks).  Timing is measured inside each
worker and printed by local rank 0 (ddp_main_torchrun.py:163-168).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def prepare():
    parser = argparse.ArgumentParser()
    parser.add_argument("--gpu", default="2,3")
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
    parser.add_argument("--checkpoint", default="ddp_checkpoint.pt")
    args = parser.parse_args()
    from ddp_practice_amd.runtime.device import select_devices

    select_devices(args.gpu)  # specify the GPUs to use
    return args


def get_ddp_generator(seed=3407):
    import torch

    local_rank = int(os.environ["LOCAL_RANK"])
    g = torch.Generator()
    g.manual_seed(seed + local_rank)
    return g


def main(args):
    import torch

    import ddp_practice_amd.distributed as dist
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import MNIST, DeviceLoader, DistributedSampler
    from ddp_practice_amd.engine import TrainLoop, evaluate
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm

    local_rank = int(os.environ["LOCAL_RANK"])
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local_rank)
    dist.init_process_group(backend="nccl" if gpu else "gloo")
    dev = torch.device("cuda", local_rank) if gpu else torch.device("cpu")
    amp = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": None}[args.amp_dtype]
    model = ConvNet(amp_dtype=amp).to(dev)
    if not args.no_sync_bn:
        model = convert_sync_batchnorm(model)
    model = DistributedDataParallel(model, device_ids=[local_rank] if gpu else None, bucket_cap_mb=args.bucket_cap_mb)
    criterion = CrossEntropyLoss().to(dev)
    optimizer = SGD(model.parameters(), 1e-4)
    scaler = GradScaler(enabled=amp is not None) if amp is not None else None
    train_dataset = MNIST(root=args.data_root, train=True, force_synthetic=args.synthetic, n=args.train_samples)
    train_sampler = DistributedSampler(train_dataset)
    g = get_ddp_generator()
    act_dtype = amp if (amp is not None and gpu) else torch.float32
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
    if local_rank == 0:
        print("begin testing", flush=True)
    correct, size = evaluate(model, test_dloader, comm=dist.default_comm(), dst=0)
    if local_rank == 0:
        print(f"Accuracy is {correct / size:.2%}", flush=True)
        state = {"model": model.state_dict()}
        if scaler is not None:
            state["scaler"] = scaler.state_dict()
        torch.save(state, args.checkpoint)
    dist.destroy_process_group()


if __name__ == "__main__":
    args = prepare()
    time_start = time.time()
    main(args)
    time_elapsed = time.time() - time_start
    if os.environ.get("LOCAL_RANK", "0") == "0":
        print(f"\ntime elapsed: {time_elapsed:.2f} seconds")
