"""A/B of the xGMI engine's remote granule pushes: system-scope relaxed atomic stores (the
default build) vs plain stores (``DPA_BUILD_TAG=pushplain DPA_EXTRA_CFLAGS=-DDPA_PUSH_PLAIN``).
W ranks share the one GPU of the box, so the 'links' are HBM: this shows what the store form
costs the kernels, not xGMI wire latency.

    python scripts/exp/push_ab.py W [label]      (DPA_EXT_SO=... selects the build)

Per size: the one-shot all-reduce (ConvNet DDP bucket 29,034 floats; SyncBN rows 65 and
1,568), the in-kernel site probe (4 workgroups, 65 floats) and the two-shot at 8 MiB;
microseconds per call from a 200-call loop between store barriers, max over ranks."""
import os
import sys
import time
from datetime import timedelta

import torch
import torch.distributed  # noqa: F401
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _bar(store, key, world):
    store.add(key, 1)
    while int(store.add(key, 0)) < world:
        time.sleep(0.0005)


def worker(rank, world, port, q):
    if world >= 3:
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
    from ddp_practice_amd import _ext
    from ddp_practice_amd.parallel.comm import open_xgmi

    _ext.load()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    store = torch.distributed.TCPStore("127.0.0.1", port, world, rank == 0, timedelta(seconds=60))
    x, err = open_xgmi(rank, world, dev, store, "p", 1 << 20, 20.0, 16 << 20)
    assert x is not None, err
    x.set_twoshot_blocks(max(8, 192 // world))
    cases = []
    for n in (65, 1568, 29034):
        t = torch.randn(n, device=dev)
        o = torch.empty_like(t)
        cases.append((f"oneshot {n}", lambda t=t, o=o: x.all_reduce(t, "sum", o), 200))
    st = torch.randn(65, device=dev)
    so = torch.empty(4 * 65, device=dev)
    cases.append(("site 65x4wg", lambda: x.site_probe(0, st, so, 4), 200))
    big = torch.randn(2 << 20, device=dev)
    bo = torch.empty_like(big)
    cases.append(("twoshot 8MiB", lambda: x.all_reduce_twoshot(big, "sum", bo), 50))
    res = {}
    for i, (name, fn, reps) in enumerate(cases):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        _bar(store, f"a{i}", world)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t0) / reps * 1e6
        assert x.error() == 0, x.error_string()
    _bar(store, "done", world)
    x.close()
    q.put((rank, res))


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    label = sys.argv[2] if len(sys.argv) > 2 else os.environ.get("DPA_EXT_SO", "default")
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
    print(f"[{label}] world {world} (ranks share one GPU): us per call, max over ranks", flush=True)
    for name in out[0]:
        print(f"  {name:16s} {max(out[r][name] for r in out):9.2f}", flush=True)


if __name__ == "__main__":
    main()
