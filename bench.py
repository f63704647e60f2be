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
        N > 1 without WORLD_SIZE in the environment: this process supervises N
        fresh rank processes (one per GPU, like the reference's mp.spawn,
        /root/reference/ddp_main.py:173-178) and never touches the GPU itself.
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
        every torchrun worker supervises ONE fresh rank process; the supervisors
        agree through torchrun's store (ddp_practice_amd/runtime/supervisor.py).

Fail-safe multi-GPU runs (N > 1):
  * every rank arms the native watchdog (DPA_BENCH_WATCHDOG s, default 90:
    no device progress / host heartbeat -> report, abort the communicator,
    exit 124) and bounds every xGMI exchange wait (DPA_XGMI_TIMEOUT, default
    15 s here); after every phase every rank reads the communicator's error word;
  * an attempt that fails (a rank exits non-zero, stalls past the attempt timeout
    DPA_BENCH_ATTEMPT_TIMEOUT (300 s), or reports a communicator error) is re-run
    by the supervisors as fresh processes with ``--comm rccl`` (no xGMI engine, no
    in-kernel exchanges; ``--share-gpu``: ``--comm host``) and the line says
    ``"fallback"`` plus the original ``comm_error``;
  * a successful ``--comm auto`` run with the xGMI engine on is followed by an A/B
    attempt on ``--comm rccl`` (headline only) -> ``ab`` keys.
  Exit status: 0 = a measured line (possibly after a fallback); 3 = every attempt
  failed (the line then has ``value`` null and ``comm_error``); 2 = bad arguments.

What one rank measures (rank 0's record becomes the JSON line):
  1. the reference's whole program on this node: 3 epochs over the 60k-sample
     train set (DistributedSampler shards, graph-replayed full batches + the
     eager tail batch) and the sharded test pass -> ``wall_3epoch_s``,
     ``epoch_img_s``, ``accuracy``; ``process_wall_3epoch_s`` adds process
     start-up (interpreter, imports, rendezvous) as the reference's timer does;
  2. the headline: exactly ``--warmup`` untimed then exactly ``--steps`` timed
     training steps, barrier + synchronize on both sides, max over ranks; then
     ``steady_img_s``: at least one full epoch of graph replays (capture excluded);
  3. the same headline in the other precisions (``value_fp16`` / ``value_fp32``:
     the reference's AMP dtype and its fp32 baseline script);
  4. the same-node baseline: the reference's step on PyTorch's own modules,
     autocast, GradScaler, SGD, SyncBatchNorm and DDP
     (ddp_practice_amd/utils/reference_step.py), same dtype -> ``vs_baseline``
     = value / baseline.  The reference's published number (other hardware,
     fp32, end to end) stays a labelled ``published_ref_img_s``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

_IMPORT_T = time.time()
ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) + 3-epoch wall-clock, MNIST ConvNet at 1/2/4/8 MI355X"
# 180,000 train images / 22.72 s (origin_main.py, 1 GPU, fp32) and / 30.82 s (ddp_main.py, W=2)
PUBLISHED_IMG_S = {1: 7923.0, 2: 5840.0}
PUBLISHED_WALL_S = {1: 22.72, 2: 30.82}
_DT = {"bf16": "bfloat16", "fp16": "float16", "fp32": None}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--amp-dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    ap.add_argument("--extra-dtypes", default="fp16,fp32",
                    help="comma list of other precisions measured the same way (value_<dt>); '' = none")
    ap.add_argument("--impl", default="native", choices=["native", "torch"],
                    help="native = this framework (headline); torch = the reference step on torch's stack")
    ap.add_argument("--steps-per-graph", type=int, default=16)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-sync-bn", action="store_true")
    ap.add_argument("--epochs", type=int, default=3, help="epochs of the measured wall-clock run (0: skip)")
    ap.add_argument("--no-steady", action="store_true", help="skip the >= 1 epoch steady-state replay timing")
    ap.add_argument("--no-baseline", action="store_true", help="skip the same-node torch baseline")
    ap.add_argument("--baseline-steps", type=int, default=200)
    ap.add_argument("--force-collectives", action="store_true",
                    help="profiling: run the DDP/SyncBN collective path even at --gpus 1")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: every rank on cuda:0, all-reduces on the xGMI engine (not the metric)")
    ap.add_argument("--comm", default=None, choices=["auto", "rccl", "xgmi", "host"],
                    help="collective algorithm selection (auto: xGMI engine where it is faster, else RCCL; "
                         "host: device tensors staged through gloo, the --share-gpu fallback)")
    ap.add_argument("--no-fallback", action="store_true", help="N > 1: report a failed attempt, do not re-run it")
    ap.add_argument("--no-ab", action="store_true", help="N > 1: skip the --comm rccl A/B attempt")
    ap.add_argument("--model", default="convnet", choices=["convnet", "resnet50"],
                    help="convnet = the headline config; resnet50 = BASELINE.json stress config 5")
    ap.add_argument("--resnet-impl", default="native", choices=["native", "torch", "torchref"],
                    help="resnet50: native NHWC kernels; torch = the torch module path with this package's "
                         "CE / GradScaler / SGD; torchref = PyTorch's own stack end to end (nn modules, "
                         "torch.autocast, F.cross_entropy, torch.optim.SGD, torch.amp.GradScaler only for fp16), "
                         "captured with torch.cuda.graph")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--train-samples", type=int, default=60000, help="synthetic train-set size (tests only)")
    ap.add_argument("--test-samples", type=int, default=10000, help="synthetic test-set size (tests only)")
    ap.add_argument("--out", default=None, help="also append the JSON line to this file")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- entry
def _spin_sync(torch, device: int):
    """hipDeviceScheduleSpin before the device's first use (runtime/device.spin_sync, opt-in
    DPA_SPIN_SYNC=1: no measured difference on the timed window).  Returns "spin", "default"
    or "spin failed: <hipError>"."""
    if torch.cuda.device_count() == 0:
        return "default"
    from ddp_practice_amd.runtime.device import spin_sync

    rc = spin_sync(device)
    return "default" if rc is None else "spin" if rc == 0 else f"spin failed: {rc}"


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    child = os.environ.get("DPA_BENCH_CHILD") == "1"
    world = int(os.environ.get("WORLD_SIZE", args.gpus))
    if not child and world > 1:
        return supervise(args, argv)
    if "WORLD_SIZE" in os.environ and not child:
        import torch

        ngpu = torch.cuda.device_count()  # does not initialise the HIP runtime on this image
        if ngpu and not args.share_gpu and int(os.environ.get("LOCAL_WORLD_SIZE", world)) > ngpu:
            print(f"bench.py: {os.environ.get('LOCAL_WORLD_SIZE', world)} local ranks but {ngpu} visible GPU(s)",
                  file=sys.stderr)
            return 2
    return run_rank(args)


# ----------------------------------------------------------------------------- supervisor (N > 1)
def _child_argv(argv: list[str], extra: list[str]) -> list[str]:
    """argv without --comm / --out (the supervisor owns them) plus ``extra``."""
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a in ("--comm", "--out"):
            skip = True
            continue
        if a.startswith("--comm=") or a.startswith("--out="):
            continue
        out.append(a)
    return [sys.executable, os.path.abspath(__file__), *out, *extra]


def _failed_record(args, n: int, err: str) -> dict:
    return {"metric": METRIC if args.model == "convnet" else
            "images/sec (whole node), ResNet-50 stress config (BASELINE.json config 5)",
            "value": None, "unit": "images/s", "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.amp_dtype, "data": "synthetic", "config": {"parallelism": f"dp{n}"},
            "comm_error": err}


def supervise(args, argv: list[str]) -> int:
    """N ranks as fresh child processes; fallback and A/B attempts (module docstring)."""
    import torch

    from ddp_practice_amd.runtime.supervisor import Supervisor, summarize

    torchrun = "WORLD_SIZE" in os.environ
    n = int(os.environ["WORLD_SIZE"]) if torchrun else args.gpus
    visible = torch.cuda.device_count()  # does not initialise the HIP runtime on this image
    if not torchrun:
        if visible == 0:
            print(f"bench.py: no GPU visible: {n} CPU ranks over gloo (plumbing only, not the metric)",
                  file=sys.stderr)
        elif not args.share_gpu and n > visible:
            print(f"bench.py: --gpus {n} but only {visible} GPU(s) are visible "
                  f"(use --share-gpu for a one-GPU rehearsal)", file=sys.stderr)
            return 2
        if args.share_gpu and visible < 1:
            print("bench.py: --share-gpu needs one visible GPU", file=sys.stderr)
            return 2
    gpu = visible > 0
    t0 = time.time()
    sup = Supervisor(n, None if torchrun else list(range(n)),
                     timeout_s=float(os.environ.get("DPA_BENCH_ATTEMPT_TIMEOUT", "300")),
                     grace_s=float(os.environ.get("DPA_BENCH_GRACE", "10")))
    env = {"DPA_BENCH_T0": repr(t0)}
    mode = args.comm or "auto"
    fb_mode = "host" if args.share_gpu else "rccl"
    attempts = []

    def attempt(m: str, extra: list[str], env_over: dict, tag: str, timeout=None):
        ta = time.time()
        res = sup.run(_child_argv(argv, ["--comm", m, *extra]), {**env, **env_over}, tag=tag, timeout_s=timeout)
        err = summarize(res)
        attempts.append({"comm": m, "tag": tag, "ok": not err, "error": err, "seconds": round(time.time() - ta, 2),
                         "xgmi_status": [(r.status or {}).get("xgmi_status") for r in res]})
        rec = (res[0].status or {}).get("record") if not err else None
        return res, err, rec

    res, err, rec = attempt(mode, [], {}, mode)
    first_err, fallback = err, None
    if err and not args.no_fallback and mode != fb_mode:
        # fresh processes; an injected fault (tests) is a one-off unless DPA_FAULT_RETRY=1
        over = {} if os.environ.get("DPA_FAULT_RETRY") == "1" else {"DPA_FAULT": ""}
        res, err, rec = attempt(fb_mode, ["--no-graph"] if fb_mode == "host" else [], over, f"fallback-{fb_mode}")
        fallback = fb_mode
    ab = None
    if (rec is not None and gpu and not args.share_gpu and not args.no_ab and mode == "auto" and fallback is None
            and args.model == "convnet" and str(rec.get("config", {}).get("comm", "")).find("xgmi on") >= 0):
        _, ab_err, ab_rec = attempt("rccl", ["--epochs", "0", "--no-baseline", "--extra-dtypes", "", "--no-steady"],
                                    {}, "ab-rccl", timeout=180)
        ab = {"auto_ms_per_step": rec.get("ms_per_step"), "auto_img_s": rec.get("value")}
        if ab_rec is not None:
            ab.update(rccl_ms_per_step=ab_rec.get("ms_per_step"), rccl_img_s=ab_rec.get("value"),
                      speedup_auto_vs_rccl=round(ab_rec["ms_per_step"] / rec["ms_per_step"], 3)
                      if rec.get("ms_per_step") else None)
        else:
            ab["rccl_error"] = ab_err
    if not sup.leader:
        return 0 if rec is not None else 3
    if rec is None:
        rec = _failed_record(args, n, err or first_err)
        rec["comm_error"] = first_err if first_err == err else f"{first_err} | fallback: {err}"
    else:
        rec["comm_error"] = first_err
    rec["fallback"] = fallback
    rec["attempts"] = attempts
    if ab is not None:
        rec["ab"] = ab
    rec["supervisor_wall_s"] = round(time.time() - t0, 2)
    _emit(rec, args.out)
    return 0 if rec.get("value") is not None else 3


# ----------------------------------------------------------------------------- helpers
def _force_collectives():
    """Profiling/rehearsal: run the DDP + SyncBN collective code path in a world of one."""
    import socket

    from ddp_practice_amd.parallel import comm as _comm

    _comm.Communicator.force_active = True
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
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


class _Health:
    """Per-rank failure detection of one bench process: the native watchdog (N > 1), the
    communicator's error word after every phase, and the status file a supervisor reads."""

    def __init__(self, comm, rank: int, world: int, gpu: bool):
        import torch

        self.comm, self.rank, self.world, self.gpu = comm, rank, world, gpu
        self.errors: dict[str, str] = {}
        self.phases: dict[str, float] = {}
        self._t = time.perf_counter()
        self.wd = None
        if world > 1:
            from ddp_practice_amd.utils import Watchdog

            self.wd = Watchdog(comm, timeout=float(os.environ.get("DPA_BENCH_WATCHDOG", "90")),
                               tag=f"bench rank{rank}")
            self.wd.heartbeat()
        self._torch = torch

    def beat(self) -> None:
        if self.wd is not None:
            self.wd.heartbeat()

    def tick(self) -> None:
        if self.wd is not None:
            self.wd.tick()

    def quiet(self) -> None:
        """A host phase of unknown length follows (library autotuning): device ticks only."""
        if self.wd is not None:
            self.wd.disarm()

    def check(self, phase: str) -> str:
        """Synchronize, then this rank's communicator error word ("" = healthy)."""
        if self.gpu:
            self._torch.cuda.synchronize()
        f = getattr(self.comm, "async_error", None)
        e = f() if f is not None else ""
        if e and e != "destroyed":
            self.errors[phase] = e
        now = time.perf_counter()
        self.phases[phase] = round(now - self._t, 4)
        self._t = now
        self.beat()
        return e

    def comm_error(self) -> str:
        return "; ".join(f"{k}: {v}" for k, v in self.errors.items())

    def finish(self, rec: dict | None, args) -> None:
        """rank 0: print the line (no supervisor) or hand it to the supervisor with the status."""
        if self.wd is not None:
            self.wd.stop()
        status_file = os.environ.get("DPA_STATUS_FILE")
        if rec is not None:
            rec["comm_error"] = self.comm_error()
            rec["phases_s"] = self.phases
        if status_file:
            st = {"rank": self.rank, "world": self.world, "comm_error": self.comm_error(),
                  "xgmi_status": getattr(self.comm, "xgmi_status", None), "comm": _comm_desc(self.comm),
                  "phases_s": self.phases, "record": rec}
            tmp = status_file + ".tmp"
            with open(tmp, "w") as f:
                json.dump(st, f)
            os.replace(tmp, status_file)
        elif rec is not None:
            _emit(rec, args.out)


class _Chunks:
    """Exactly ``n`` training steps as replays of a K-step graph plus one graph of the remainder,
    keeping the loader's device step counter inside the epoch's full batches."""

    def __init__(self, step, spg: int, loader, nfull: int, graphs: bool, health: _Health | None = None):
        from ddp_practice_amd.runtime import CapturedStep

        self.step, self.spg, self.loader, self.nfull = step, max(1, spg), loader, nfull
        self.graphs = graphs
        self.health = health
        self._mk = lambda k: CapturedStep(step, warmup=2, steps_per_graph=k, enabled=graphs,
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

    def _plan(self, n: int) -> list:
        """Chunk sizes of ``run(n)``: a one-step graph first (the device starts after ~6 node
        submissions instead of a whole graph's: r5y measured ~25 us of device idle in a 20-step
        window), then the remainder, then full graphs -- the host submits each next graph while
        the device runs the previous one.  DPA_BENCH_LEAD=0: remainder first, no lead step."""
        if n <= 0:
            return []
        if self.spg > 1 and os.environ.get("DPA_BENCH_PLAN") == "geo":
            # A/B: 1, 2, 4, ... steps per graph (capped at spg), each next graph submitted while
            # the device runs the previous one: no gain -- the device span of the 20-step window
            # is already 20 steady steps; the fixed cost is launch / sync latency outside it
            # (profiles/r6av_window_plan_ab.txt)
            plan, k, left = [], 1, n
            while left > 0:
                c = min(k, self.spg, left)
                plan.append(c)
                left -= c
                k *= 2
            return plan
        lead = 1 if (self.spg > 1 and os.environ.get("DPA_BENCH_LEAD") != "0") else 0
        m = n - lead
        plan = [lead] if lead else []
        if m % self.spg:
            plan.append(m % self.spg)
        plan += [self.spg] * (m // self.spg)
        return plan

    def prepare(self, n: int) -> None:
        """Capture every graph ``run(n)`` needs (outside any timed region)."""
        for k in sorted(set(self._plan(n))):
            self.runner(k)

    def _chunk(self, k: int) -> None:
        if self.pos + k > self.nfull:
            self.loader.set_step(0)
            self.pos = 0
        self.runners[k].run()
        self.pos += k

    def run(self, n: int) -> None:
        tick = self.health.tick if self.health is not None else None
        for i, k in enumerate(self._plan(n)):
            self._chunk(k)
            if tick is not None and i % 64 == 63:
                tick()
        if tick is not None:
            tick()


# ----------------------------------------------------------------------------- ConvNet
def run_rank(args) -> int:
    if args.model == "resnet50":
        return bench_resnet(args)
    t_proc0 = _process_t0()
    marks = {"bench_imported": round(_IMPORT_T - t_proc0, 3)}
    import torch

    marks["torch_imported"] = round(time.time() - t_proc0, 3)
    from ddp_practice_amd import distributed as ddist
    from ddp_practice_amd.data import synthetic

    marks["package_imported"] = round(time.time() - t_proc0, 3)

    if args.comm:
        os.environ["DPA_COMM"] = args.comm
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.share_gpu:  # ranks share one device (ops/convnet_fused.py; one HW queue each at 3+)
        from ddp_practice_amd.runtime.device import shared_cu_mask, shared_gpu_env

        shared_gpu_env(world)  # before the first HIP call below
        shared_cu_mask(world, int(os.environ.get("RANK", "0")))
    local_rank = 0 if args.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    spin_rc = _spin_sync(torch, local_rank)  # opt-in busy-polled host waits (runtime/device.spin_sync)
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
    else:  # CPU plumbing (BASELINE config 1): torch modules, gloo, no graphs, fp32
        dev = torch.device("cpu")
        args.no_graph, args.no_baseline, args.amp_dtype, args.extra_dtypes = True, True, "fp32", ""

    dist_path = world > 1 or args.force_collectives
    if args.force_collectives:
        _force_collectives()
    if world > 1:
        # a stalled exchange must end well inside the driver's timeout (default 600 s in the engine)
        os.environ.setdefault("DPA_XGMI_TIMEOUT", "15")
    if dist_path:
        if not gpu:
            backend = "gloo"
        elif args.comm == "host":
            backend = "host"
        else:
            backend = "xgmi" if args.share_gpu else "nccl"
        ddist.init_process_group(backend=backend)
    comm = ddist.default_comm()
    rank = ddist.get_rank()
    health = _Health(comm, rank, world, gpu)
    marks["comm_ready"] = round(time.time() - t_proc0, 3)
    # the synthetic sets are generated in HBM by one kernel (host numpy on CPU): data/mnist.py
    train_ds = synthetic(args.train_samples, seed=1, name="synthetic-MNIST-train", device=dev)
    test_ds = synthetic(args.test_samples, seed=2, name="synthetic-MNIST-test", device=dev)
    marks["data_ready"] = round(time.time() - t_proc0, 3)
    health.check("setup")
    B = args.batch_size
    ctx = dict(args=args, world=world, rank=rank, dev=dev, gpu=gpu, dist_path=dist_path, local_rank=local_rank,
               comm=comm, train_ds=train_ds, test_ds=test_ds, health=health, marks=marks, t_proc0=t_proc0)
    rec_extra: dict = {}

    # 1. the reference's program: 3 epochs + sharded test, measured end to end
    if args.epochs > 0 and args.impl == "native":
        rec_extra.update(_three_epochs(ctx))
        health.check("3epoch")

    # 2. the headline: exactly K timed steps after exactly W warm-up steps (+ steady state)
    amp = _amp(args.amp_dtype)
    if args.impl == "native":
        h = _headline(ctx, amp, steady=not args.no_steady)
    else:
        h = _torch_headline(ctx, amp)
    health.check("headline")
    ms, img_s = h["ms"], h["img_s"]
    if "steady_img_s" in h:
        rec_extra.update(steady_img_s=h["steady_img_s"], steady_ms_per_step=h["steady_ms"],
                         steady_steps=h["steady_steps"])

    # 3. the other precisions, same steps / warm-up
    for dt in [d for d in args.extra_dtypes.split(",") if d and d != args.amp_dtype]:
        if args.impl != "native":
            break
        try:
            x = _headline(ctx, _amp(dt), steady=not args.no_steady)
            rec_extra[f"value_{dt}"] = round(x["img_s"], 1)
            rec_extra[f"ms_per_step_{dt}"] = round(x["ms"], 5)
            if "steady_img_s" in x:
                rec_extra[f"steady_img_s_{dt}"] = x["steady_img_s"]
        except Exception as e:  # noqa: BLE001 - context keys, never the metric
            rec_extra[f"error_{dt}"] = f"{type(e).__name__}: {e}"
        health.check(f"headline_{dt}")

    # 4. same-node baseline: the reference step on torch's own stack, same dtype
    base = None
    if args.impl == "native" and not args.no_baseline and not args.share_gpu:
        health.quiet()  # torch's first convolutions may autotune for a while: device ticks only
        try:
            from ddp_practice_amd.utils.reference_step import TorchReferenceStep
            from ddp_practice_amd.data import DistributedSampler

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
        health.check("baseline")
    elif args.share_gpu:
        rec_extra["baseline_error"] = "skipped: --share-gpu rehearsal"

    seen = _ranks_seen(comm if dist_path else None)
    health.check("end")
    rec = None
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
                "impl": h["impl"],
                "sync_bn": dist_path and not args.no_sync_bn,
                "amp": f"autocast {args.amp_dtype} + GradScaler" if amp is not None else "fp32",
                "optimizer": "SGD(lr=1e-4)",
                "hipgraph": bool(h["captured"]), "host_wait": spin_rc,
                "steps_per_graph": h["spg"],
                "comm": _comm_desc(comm) if dist_path else "none (1 rank)",
                "grad_avg": h["grad_avg"],
                "shared_gpu": bool(args.share_gpu),
            },
            "ranks_seen": seen,
            "per_rank_max_s": round(h["dt"], 6),
        }
        rec.update(rec_extra)
    health.finish(rec, args)
    ddist.destroy_process_group()
    return 0


def _amp(name: str):
    import torch

    return {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[name]


def _build(ctx, amp, seed: int):
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.models import ConvNet
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm
    import torch

    torch.manual_seed(seed)
    model = ConvNet(amp_dtype=amp).to(ctx["dev"])
    if ctx["dist_path"]:
        if not ctx["args"].no_sync_bn:
            model = convert_sync_batchnorm(model)
        model = DistributedDataParallel(model, device_ids=[ctx["local_rank"]] if ctx["gpu"] else None,
                                        gradient_as_bucket_view=True)
    return model, SGD(model.parameters(), lr=1e-4), GradScaler(enabled=amp is not None)


def _three_epochs(ctx) -> dict:
    import torch

    from ddp_practice_amd import distributed as ddist
    from ddp_practice_amd.data import DeviceLoader, DistributedSampler
    from ddp_practice_amd.engine import TrainLoop, evaluate
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.utils import FaultInjector

    args, world, rank, dev, comm, health = (ctx[k] for k in ("args", "world", "rank", "dev", "comm", "health"))
    amp = _amp(args.amp_dtype)
    act = amp if amp is not None else torch.float32
    train_ds, test_ds = ctx["train_ds"], ctx["test_ds"]
    B = args.batch_size
    model, opt, scaler = _build(ctx, amp, 0)
    g = torch.Generator()
    g.manual_seed(3407 + rank)
    tr = DeviceLoader(train_ds, batch_size=B, sampler=DistributedSampler(train_ds, num_replicas=world, rank=rank),
                      generator=g, device=dev, dtype=act)
    te = DeviceLoader(test_ds, batch_size=B, sampler=DistributedSampler(test_ds, num_replicas=world, rank=rank),
                      device=dev, dtype=act)
    loop = TrainLoop(model, CrossEntropyLoss().to(dev), opt, tr, scaler if amp is not None else None,
                     use_graph=not args.no_graph, steps_per_graph=args.steps_per_graph,
                     watchdog=health.wd, faults=FaultInjector(rank))

    def sync():
        if ctx["gpu"]:
            torch.cuda.synchronize()

    ddist.barrier()
    sync()
    ctx["marks"]["3epoch_start"] = round(time.time() - ctx["t_proc0"], 3)
    t0 = time.perf_counter()
    for ep in range(args.epochs):
        tr.sampler.set_epoch(ep)
        loop.run_epoch()
        health.beat()
    sync()
    t_train = time.perf_counter() - t0
    correct, size = evaluate(model, te, comm=comm if comm.active else None, dst=0)
    sync()
    ddist.barrier()
    t_all = time.perf_counter() - t0
    t_proc = time.time() - _process_t0()
    t_train, t_all, t_proc = (ddist.max_over_ranks(v) for v in (t_train, t_all, t_proc))
    imgs = args.epochs * len(train_ds)
    out = {
        "wall_3epoch_s": round(t_all, 3),
        "process_wall_3epoch_s": round(t_proc, 3),
        "epoch_img_s": round(imgs / t_train, 1),
        "train_3epoch_s": round(t_train, 3),
        "epochs": args.epochs,
        "accuracy": round(correct / size, 4) if rank == 0 and size else None,
        "steps_per_rank_per_epoch": len(tr),
        "published_ref_wall_s": PUBLISHED_WALL_S.get(world),
    }
    if loop.graph_error is not None:
        out["graph_error_3epoch"] = repr(loop.graph_error)
    ctx["marks"]["3epoch_end"] = round(time.time() - ctx["t_proc0"], 3)
    out["startup_marks_s"] = ctx["marks"]
    return out


def _headline(ctx, amp, steady: bool) -> dict:
    """Exactly --warmup untimed + --steps timed steps of the native step (graph replays),
    then (``steady``) at least one full epoch of replays timed the same way."""
    import torch

    from ddp_practice_amd import distributed as ddist
    from ddp_practice_amd.data import DeviceLoader, DistributedSampler, accepts_deferred
    from ddp_practice_amd.nn import CrossEntropyLoss

    args, world, rank, dev, health = (ctx[k] for k in ("args", "world", "rank", "dev", "health"))
    B = args.batch_size
    act = amp if amp is not None else torch.float32
    train_ds = ctx["train_ds"]
    model, optimizer, scaler = _build(ctx, amp, 1)
    crit = CrossEntropyLoss().to(dev)
    # the fused optimizer launch: the AMP step, or fp32's plain step (optim/sgd.py)
    fusable = amp is not None or getattr(optimizer, "plain_fused", False)
    fused_grad = ctx["dist_path"] and fusable and model.defer_grad_sync_to(optimizer)
    # conv1's weight-gradient column sums run inside the fused step (engine.TrainLoop does the
    # same): without DDP, and under DDP when the step also averages the gradients (fused_grad)
    if fusable and (fused_grad or not ctx["dist_path"]):
        model.set_slab_sink(optimizer)
    sampler = DistributedSampler(train_ds, num_replicas=world, rank=rank)
    loader = DeviceLoader(train_ds, batch_size=B, sampler=sampler, device=dev, dtype=act)
    images, labels = loader.static_batch()
    loader.start_epoch()
    nfull = len(sampler) // B
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

    spg = 1 if args.no_graph else args.steps_per_graph
    chunks = _Chunks(step, spg, loader, nfull, graphs=not args.no_graph, health=health)
    n_steady = max(nfull, args.steps) if steady else 0
    for n in (args.warmup, args.steps, n_steady):
        if n:
            chunks.prepare(n)
    if chunks.capture_error is not None and rank == 0:
        print(f"[bench] graph capture failed, eager fallback: {chunks.capture_error!r}", file=sys.stderr)

    ev = ctx["gpu"] and os.environ.get("DPA_BENCH_EVENTS") == "1"  # diagnostics: device-side span

    def timed(n: int) -> float:
        ddist.barrier()
        if ctx["gpu"]:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        if ev:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        chunks.run(n)
        if ev:
            e1.record()
            th = time.perf_counter() - t0
        if ctx["gpu"]:
            torch.cuda.synchronize()
        ddist.barrier()
        dt = time.perf_counter() - t0
        if ev:
            print(f"[bench] {n} steps: wall {dt * 1e6:.1f} us, device span {e0.elapsed_time(e1) * 1e3:.1f} us, "
                  f"host issue {th * 1e6:.1f} us", file=sys.stderr)
        return ddist.max_over_ranks(dt)

    chunks.run(args.warmup)
    dt = timed(args.steps)
    out = {"dt": dt, "ms": dt / args.steps * 1e3, "img_s": B * world * args.steps / dt,
           "captured": chunks.graphs and chunks.capture_error is None, "spg": spg,
           "impl": "native (fused HIP kernels, C++ reducer/communicator)" if ctx["gpu"] else
                   "CPU plumbing (torch modules, gloo; not the metric)",
           "grad_avg": ("in AMP-SGD kernel (xGMI)" if fused_grad else "reducer all-reduce") if ctx["dist_path"]
                       else "none (1 rank)"}
    if n_steady:
        ds = timed(n_steady)
        out.update(steady_img_s=round(B * world * n_steady / ds, 1), steady_ms=round(ds / n_steady * 1e3, 5),
                   steady_steps=n_steady)
    del chunks, model, optimizer, scaler, loader
    return out


def _torch_headline(ctx, amp) -> dict:
    from ddp_practice_amd import distributed as ddist
    from ddp_practice_amd.data import DistributedSampler
    from ddp_practice_amd.utils.reference_step import TorchReferenceStep

    args, world, rank, dev = (ctx[k] for k in ("args", "world", "rank", "dev"))
    train_ds = ctx["train_ds"]
    ref = TorchReferenceStep(dev, amp, world, *train_ds.to_device(dev),
                             DistributedSampler(train_ds, num_replicas=world, rank=rank).indices().to(dev),
                             args.batch_size, local_rank=ctx["local_rank"], seed=1)
    dt = ddist.max_over_ranks(ref.time_steps(args.steps, args.warmup, ddist.barrier))
    return {"dt": dt, "ms": dt / args.steps * 1e3, "img_s": args.batch_size * world * args.steps / dt,
            "captured": False, "spg": 1,
            "impl": "torch (nn modules, torch.autocast, torch GradScaler/SGD/SyncBatchNorm/DDP)",
            "grad_avg": "torch DDP" if world > 1 else "none (1 rank)"}


# ----------------------------------------------------------------------------- ResNet-50
def _torchref_resnet_step(model, images, labels, amp, lr: float):
    """PyTorch's own ResNet-50 training step, captured with ``torch.cuda.graph`` (the
    library bar for the native path, VERDICT r3 Weak 5).  bf16: no GradScaler (torch's
    recommendation: bf16 has fp32's range, and ``GradScaler.step`` syncs the host through
    ``found_inf.item()``, which no graph can capture); fp16 keeps the scaler and runs
    eagerly.  Warm-up and capture run on a side stream (torch.cuda.graph's contract: the
    AccumulateGrad nodes then live on the capture stream).  Returns (run, captured, why)."""
    import torch
    import torch.nn.functional as F

    opt = torch.optim.SGD(model.parameters(), lr=lr, foreach=True)
    scaler = torch.amp.GradScaler("cuda") if amp == torch.float16 else None

    def step():
        with torch.autocast("cuda", dtype=amp, enabled=amp is not None):
            out = model(images)
        loss = F.cross_entropy(out, labels)
        if scaler is not None:
            opt.zero_grad(set_to_none=True)
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()
        else:
            opt.zero_grad(set_to_none=False)
            loss.backward()
            opt.step()

    if scaler is not None:
        return step, False, "fp16 GradScaler.step syncs the host (found_inf.item())"
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    from ddp_practice_amd.runtime.graph import gc_paused

    try:
        with gc_paused(), torch.cuda.graph(g):
            step()
    except Exception as e:  # noqa: BLE001 - reported in the JSON line, eager fallback
        torch.cuda.synchronize()
        return step, False, f"{type(e).__name__}: {str(e).splitlines()[0]}"
    return g.replay, True, ""


def bench_resnet(args) -> int:
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
    if args.share_gpu:  # ranks share one device (runtime/device.py)
        from ddp_practice_amd.runtime.device import shared_cu_mask, shared_gpu_env

        # 4 HIP queues per rank, not the one-queue default from 3 ranks: with one queue every
        # rank segfaulted inside hipGraphLaunch at the first replay of the ResNet-50 step
        # graph (profiles/r6ag_resnet50_share_w4_q1_segv.txt; 4 queues: r6ah, r6ai)
        os.environ.setdefault("DPA_SHARED_HW_QUEUES", "4")
        shared_gpu_env(world)
        shared_cu_mask(world, int(os.environ.get("RANK", "0")))
    spin_rc = _spin_sync(torch, local_rank)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    dist_path = world > 1 or args.force_collectives
    if args.force_collectives:
        _force_collectives()
    if world > 1:
        os.environ.setdefault("DPA_XGMI_TIMEOUT", "15")
    if dist_path:
        ddist.init_process_group(backend="host" if args.comm == "host" else "xgmi" if args.share_gpu else "nccl")
    rank = ddist.get_rank()
    c = ddist.default_comm()
    health = _Health(c, rank, world, True)
    amp = _amp(args.amp_dtype)
    bs = args.batch_size if args.batch_size != 32 else 128
    torch.manual_seed(0)
    torchref = args.resnet_impl == "torchref"
    model = resnet50(amp_dtype=None if torchref else amp, fused=args.resnet_impl == "native").to(dev)
    if args.resnet_impl != "native":
        model = model.to(memory_format=torch.channels_last)
    if dist_path and torchref:
        raise SystemExit("--resnet-impl torchref: one GPU only (the library bar of the single-rank step)")
    if dist_path:
        if not args.no_sync_bn:
            model = convert_sync_batchnorm(model)
        model = DistributedDataParallel(model, device_ids=[local_rank], gradient_as_bucket_view=True)
    optimizer = SGD(model.parameters(), lr=1e-4)
    scaler = GradScaler(enabled=amp is not None)
    g = torch.Generator(device="cpu").manual_seed(rank)
    images = torch.rand(bs, 3, args.image_size, args.image_size, generator=g).to(dev)
    labels = torch.randint(0, 1000, (bs,), generator=g).to(dev)
    if args.resnet_impl != "native":
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
    health.quiet()
    capture_note = ""
    if torchref:
        run, captured, capture_note = _torchref_resnet_step(model, images, labels, amp, 1e-4)
        if args.no_graph:
            captured = False
        if not captured and rank == 0:
            print(f"[bench] torchref eager: {capture_note}", file=sys.stderr)

        class _R:
            pass

        runner = _R()
        runner.run = run
    else:
        runner = CapturedStep(step, warmup=2, steps_per_graph=1, enabled=not args.no_graph)
        captured = runner.capture() if not args.no_graph else False
        if not captured and not args.no_graph:
            capture_note = repr(runner.capture_error)
            if rank == 0:
                print(f"[bench] graph capture failed, eager: {capture_note}", file=sys.stderr)
    health.check("setup")
    for _ in range(args.warmup):
        runner.run()
    ddist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner.run()
        health.tick()
    torch.cuda.synchronize()
    ddist.barrier()
    dt = ddist.max_over_ranks(time.perf_counter() - t0)
    health.check("headline")
    ms = dt / args.steps * 1e3
    img_s = bs * world * args.steps / dt
    seen = _ranks_seen(c if dist_path else None)
    rec = None
    if rank == 0:
        rec = {
            "metric": "images/sec (whole node), ResNet-50 stress config (BASELINE.json config 5)",
            "value": round(img_s, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.amp_dtype,
            "data": f"synthetic 3x{args.image_size}x{args.image_size}, random-init weights",
            "config": {"model": "ResNet-50 (25,557,032 params)", "global_batch": bs * world, "seq_len": None,
                       "parallelism": f"dp{world}", "per_rank_batch": bs, "impl": args.resnet_impl,
                       "sync_bn": dist_path and not args.no_sync_bn, "optimizer": "SGD(lr=1e-4)",
                       "comm": _comm_desc(c) if dist_path else "none", "hipgraph": bool(captured), "host_wait": spin_rc,
                       "shared_gpu": bool(args.share_gpu),
                       "stack": ("torch nn + torch.autocast + F.cross_entropy + torch.optim.SGD(foreach)"
                                 + (" + torch.amp.GradScaler" if amp == torch.float16 else " (bf16: no GradScaler)")
                                 if torchref else "this package's CE / GradScaler / SGD")},
            "capture_note": capture_note,
            "ranks_seen": seen, "per_rank_max_s": round(dt, 6),
        }
    health.finish(rec, args)
    ddist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
