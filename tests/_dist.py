"""Multi-process helpers for CPU (gloo) distributed tests."""
import os
import socket
import traceback

import torch
import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    torch.set_num_threads(2)
    try:
        import ddp_practice_amd.distributed as dist

        dist.init_process_group("gloo")
        out = fn(rank, world, *args)
        dist.destroy_process_group()
        q.put((rank, "ok", out))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))


def run(fn, world=2, args=(), timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, st, out = q.get(timeout=timeout)
            if st != "ok":
                raise AssertionError(f"rank {rank} failed:\n{out}")
            res[rank] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [res[r] for r in range(world)]
