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
Extra flags: --synthetic, --data-root, --amp-dtype, --no-graph, --seed,
--checkpoint.
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
    parser.add_argument("--data-root", default="./data")
    parser.add_argument("--synthetic", action="store_true", help="use the synthetic MNIST-shaped dataset")
    parser.add_argument("--train-samples", type=int, default=None, help="synthetic train-set size (tests)")
    parser.add_argument("--test-samples", type=int, default=None, help="synthetic test-set size (tests)")
    parser.add_argument("--amp-dtype", default="fp32", choices=["fp32", "bf16", "fp16"])
    parser.add_argument("--no-graph", action="store_true", help="run the training step eagerly")
    parser.add_argument("--seed", type=int, default=None)
    parser.add_argument("--checkpoint", default="origin_checkpoint.pt")
    args = parser.parse_args()
    from ddp_practice_amd.runtime.device import select_devices

    select_devices(args.gpu)  # before any HIP initialisation
    return args


def main(args):
    import torch

    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import MNIST, DeviceLoader
    from ddp_practice_amd.engine import TrainLoop, evaluate
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD

    if args.seed is not None:
        torch.manual_seed(args.seed)
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    amp = {"fp32": None, "bf16": torch.bfloat16, "fp16": torch.float16}[args.amp_dtype]
    model = ConvNet(amp_dtype=amp).to(dev)
    criterion = CrossEntropyLoss().to(dev)
    optimizer = SGD(model.parameters(), 1e-4)
    scaler = GradScaler(enabled=amp is not None) if amp is not None else None
    train_dataset = MNIST(root=args.data_root, train=True, force_synthetic=args.synthetic, n=args.train_samples)
    test_dataset = MNIST(root=args.data_root, train=False, force_synthetic=args.synthetic, n=args.test_samples)
    act_dtype = amp if (amp is not None and dev.type == "cuda") else torch.float32
    train_dloader = DeviceLoader(train_dataset, batch_size=args.batch_size, shuffle=True, device=dev,
                                 dtype=act_dtype, num_workers=4, pin_memory=True)
    test_dloader = DeviceLoader(test_dataset, batch_size=args.batch_size, shuffle=True, device=dev,
                                dtype=act_dtype, num_workers=2, pin_memory=True)
    loop = TrainLoop(model, criterion, optimizer, train_dloader, scaler, use_graph=not args.no_graph)
    for epoch in range(args.epochs):
        print(f"begin training of epoch {epoch + 1}/{args.epochs}")
        loop.run_epoch()
    if loop.graph_error is not None:
        print(f"[ddp_practice_amd] hipGraph capture failed, ran eagerly: {loop.graph_error!r}", file=sys.stderr)
    print("begin testing")
    correct, size = evaluate(model, test_dloader)
    print(f"Accuracy is {correct / size:.2%}")
    torch.save({"model": model.state_dict()}, args.checkpoint)


if __name__ == "__main__":
    args = prepare()
    time_start = time.time()
    main(args)
    time_elapsed = time.time() - time_start
    print(f"\ntime elapsed: {time_elapsed:.2f} seconds")
