"""W ranks sharing the one GPU of the box: all-reduce timings of the xGMI engine's
two-shot (reduce-scatter + all-gather) vs the chunked one-shot, at DDP-bucket sizes.
(Peers on one device: the 'links' are HBM, so this shows the paths run and their
relative cost, not xGMI bandwidth.)   python scripts/exp/xgmi_rehearsal.py W"""
import os
import sys
import time
from datetime import timedelta

import torch
import torch.distributed  # noqa: F401
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def worker(rank, world, port, q):
    from ddp_practice_amd import _ext
    from ddp_practice_amd.parallel.comm import open_xgmi

    C = _ext.load()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    store = torch.distributed.TCPStore("127.0.0.1", port, world, rank == 0, timedelta(seconds=60))
    # one-shot chunk: every rank's one-shot grid (chunk / 8 KB workgroups) must be resident
    # together on the shared GPU -> 1 MiB chunks (128 workgroups per rank)
    x, err = open_xgmi(rank, world, dev, store, "r", 1 << 20, 20.0, 32 << 20)
    assert x is not None, err
    x.set_twoshot_blocks(max(8, 192 // world))
    xc = C.xgmi.XgmiCollective(x)
    rows = []
    for mib in (1, 8, 25):
        n = mib * (1 << 20) // 4
        t = torch.randn(n, device=dev)
        res = {}
        for name, fn in (("two-shot", lambda: x.all_reduce_twoshot(t)),
                         ("one-shot chunks", lambda: [x.all_reduce(c) for c in t.split((1 << 20) // 4)])):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            store.add(f"b{mib}{name}", 1)
            while int(store.add(f"b{mib}{name}", 0)) < world:
                time.sleep(0.001)
            t0 = time.perf_counter()
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            res[name] = (time.perf_counter() - t0) / 10 * 1e3
        assert x.error() == 0, x.error_string()
        rows.append((mib, res["two-shot"], res["one-shot chunks"]))
    xc.all_reduce(torch.ones(8 << 20, device=dev))  # > one-shot size: the collective routes to two-shot
    torch.cuda.synchronize()
    store.add("done", 1)
    while int(store.add("done", 0)) < world:
        time.sleep(0.001)
    x.close()
    q.put((rank, rows))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    from tests._dist import free_port

    port = free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(60)
    print(f"world {world} (ranks share one GPU): all-reduce ms, max over ranks")
    print(f"{'MiB':>5s} {'two-shot':>10s} {'one-shot chunks':>16s}")
    for i, (mib, _, _) in enumerate(out[0]):
        ts = max(out[r][i][1] for r in out)
        os_ = max(out[r][i][2] for r in out)
        print(f"{mib:5d} {ts:10.3f} {os_:16.3f}")


if __name__ == "__main__":
    main()
