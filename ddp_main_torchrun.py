"""DDP + SyncBN + AMP ConvNet training launched by torchrun.

Same CLI and behaviour as /root/reference/ddp_main_torchrun.py:
    torchrun --standalone --nproc_per_node=2 ddp_main_torchrun.py --gpu 0,1
The elastic agent provides RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT; ``init_process_group("nccl")`` uses env://.  ``--gpu`` sets
CUDA_VISIBLE_DEVICES as in the reference (whose default "2,3" needs a 4+ GPU
node — pass ``--gpu 0,...,N-1`` for N ranks).  Timing is measured inside each
worker and printed by local rank 0 (ddp_main_torchrun.py:163-168).
Additive flags: see ddp_practice_amd/cli.py.
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
    from ddp_practice_amd.cli import add_run_args

    add_run_args(parser, amp_default="fp16", checkpoint="ddp_checkpoint.pt", distributed=True)
    args = parser.parse_args()
    from ddp_practice_amd.cli import apply_env

    apply_env(args)
    from ddp_practice_amd.runtime.device import select_devices

    select_devices(args.gpu.split(",")[0] if args.share_gpu else args.gpu)  # specify the GPUs to use
    return args


def main(args):
    import torch

    import ddp_practice_amd.distributed as dist
    from ddp_practice_amd.cli import dist_backend, rank_device_index, run, share_gpu_rank_env

    local_rank = int(os.environ["LOCAL_RANK"])
    share_gpu_rank_env(args, local_rank)
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(rank_device_index(args, local_rank))
    dist.init_process_group(backend=dist_backend(args) if gpu else "gloo")
    run(args, distributed=True, local_rank=local_rank, generator_seed=3407 + local_rank)


if __name__ == "__main__":
    args = prepare()
    time_start = time.time()
    main(args)
    time_elapsed = time.time() - time_start
    if os.environ.get("LOCAL_RANK", "0") == "0":
        print(f"\ntime elapsed: {time_elapsed:.2f} seconds")
