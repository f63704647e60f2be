"""Single-process ConvNet training (fp32) — the reference baseline, MI355X-native.

Same CLI, stdout and checkpoint as /root/reference/origin_main.py:
    python origin_main.py --gpu 0 [-e 3] [-b 32]
prints ``begin training of epoch e/E``, ``begin testing``, ``Accuracy is xx.xx%``
and ``time elapsed: X.XX seconds`` and writes ``origin_checkpoint.pt`` =
``{"model": state_dict}``.

Differences by design (see README): ``--gpu`` is applied (the reference parses
but ignores it, origin_main.py:36); the dataset lives in HBM and batches are
gathered on the device; on a GPU the training step is replayed from a hipGraph.
Without a GPU it runs the same loop on CPU (BASELINE config 1, plumbing).
Additive flags: see ddp_practice_amd/cli.py.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def prepare():
    parser = argparse.ArgumentParser()
    parser.add_argument("--gpu", default="0")
    parser.add_argument("-e", "--epochs", default=3, type=int, metavar="N", help="number of total epochs to run")
    parser.add_argument("-b", "--batch_size", default=32, type=int, metavar="N", help="number of batchsize")
    from ddp_practice_amd.cli import add_run_args

    add_run_args(parser, amp_default="fp32", checkpoint="origin_checkpoint.pt", distributed=False)
    args = parser.parse_args()
    from ddp_practice_amd.runtime.device import select_devices

    select_devices(args.gpu)  # before any HIP initialisation
    return args


def main(args):
    from ddp_practice_amd.cli import run

    run(args, distributed=False)


if __name__ == "__main__":
    args = prepare()
    time_start = time.time()
    main(args)
    time_elapsed = time.time() - time_start
    print(f"\ntime elapsed: {time_elapsed:.2f} seconds")
