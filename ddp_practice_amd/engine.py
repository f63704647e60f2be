"""Training / evaluation loops shared by the CLIs and the benchmark.

The per-batch semantics are the reference's
(/root/reference/ddp_main.py:83-93 ``train`` and :96-112 ``test``):

    outputs = model(images); loss = criterion(outputs, labels)
    optimizer.zero_grad(); scaler.scale(loss).backward()
    scaler.step(optimizer); scaler.update()

On a HIP device the step for full batches is captured once into a hipGraph
(``runtime.CapturedStep``) and replayed; the batch position lives in a device
counter advanced by the gather kernel, so an epoch is ``n_full / K`` graph
replays plus (if the sampler leaves one) a partial last batch run eagerly.
The warm-up iteration that capture needs is undone (model, buffers,
optimizer and scaler state are snapshotted and restored), so the sequence of
optimizer steps is exactly the reference's.  On CPU the same loop runs eagerly.
"""
from __future__ import annotations

import contextlib

import torch

from .data.loader import DeviceLoader
from .runtime.graph import CapturedStep
from .utils.trace import trace_range


def _snapshot(model, optimizer, scaler):
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    opt = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in st.items()}
           for p, st in optimizer.state.items()}
    sc = None
    if scaler is not None and getattr(scaler, "_scale", None) is not None:
        sc = (scaler._scale.clone(), scaler._growth_tracker.clone(), scaler._found_inf.clone())
    return sd, opt, sc


def _restore(model, optimizer, scaler, snap):
    sd, opt, sc = snap
    with torch.no_grad():
        for k, v in model.state_dict().items():
            v.copy_(sd[k])
    for p in list(optimizer.state.keys()):
        if id(p) in opt:
            for k, v in opt[id(p)].items():
                if torch.is_tensor(v):
                    optimizer.state[p][k].copy_(v)
                else:
                    optimizer.state[p][k] = v
        else:
            # state created by the warm-up step: keep the tensors (a captured graph
            # may reference them) but reset them
            for k, v in optimizer.state[p].items():
                if torch.is_tensor(v):
                    v.zero_()
    if sc is not None:
        scaler._scale.copy_(sc[0])
        scaler._growth_tracker.copy_(sc[1])
        scaler._found_inf.copy_(sc[2])


class TrainLoop:
    """Epoch runner: graph-replayed full batches + eager tail batch."""

    def __init__(self, model, criterion, optimizer, loader: DeviceLoader, scaler=None, use_graph: bool = True,
                 steps_per_graph: int = 16, watchdog=None, faults=None):
        self.model = model
        self.criterion = criterion
        self.optimizer = optimizer
        self.loader = loader
        self.scaler = scaler
        self.device = loader.device
        self.use_graph = use_graph and self.device.type == "cuda"
        self.spg = max(1, steps_per_graph)
        self.images, self.labels = loader.static_batch()
        self._graphs: dict[int, CapturedStep] = {}
        self.graph_error = None
        self.watchdog = watchdog  # utils.Watchdog: ticked after every chunk of steps
        self.faults = faults if faults else None  # utils.FaultInjector (DPA_FAULT)
        # DDP + fused AMP step: the optimizer kernel averages the gradients over xGMI
        # (parallel/ddp.py defer_grad_sync_to; a no-op without the engine)
        # (fp32 without a scaler: the optimizer's plain step is the same fused launch, optim/sgd.py)
        fused = (getattr(scaler, "_enabled", False) if scaler is not None
                 else getattr(optimizer, "plain_fused", False))
        if fused and hasattr(model, "defer_grad_sync_to"):
            if model.defer_grad_sync_to(optimizer):
                model.set_slab_sink(optimizer)  # and the conv1 slab sums (exchanged in the same launch)
        elif fused and hasattr(model, "set_slab_sink"):
            # no DDP: the fused step also sums the conv1 weight-gradient slab (models/convnet.py)
            model.set_slab_sink(optimizer)
        self.global_step = 0
        # the model's first kernel gathers the batch itself (no gather launch per step)
        from .data.loader import accepts_deferred

        self._defer = accepts_deferred(model, self.images)

    # -- one step on the static buffers (what gets captured)
    def _step(self, images=None, labels=None, fill=True, before_update=None):
        if fill:
            self.loader.fill_(self.images, self.labels, defer=self._defer)
        images = self.images if images is None else images
        labels = self.labels if labels is None else labels
        with trace_range("forward"):
            outputs = self.model(images)
            loss = self.criterion(outputs, labels)
        self.optimizer.zero_grad(set_to_none=True)
        if self.scaler is not None:
            with trace_range("backward"):
                self.scaler.scale(loss).backward()
            if before_update is not None:
                flush = getattr(self.optimizer, "_flush_deferred", None)
                if flush is not None:
                    flush()  # the hook reads .grad
                before_update()
            with trace_range("optimizer"):
                self.scaler.step(self.optimizer)
                self.scaler.update()
        else:
            with trace_range("backward"):
                loss.backward()
            if before_update is not None:
                before_update()
            with trace_range("optimizer"):
                self.optimizer.step()
        return loss

    def _eager_step(self, images=None, labels=None, fill=True):
        """One un-captured step (CPU, tail batches, steps with an injected fault)."""
        step = self.global_step
        hook = None
        if self.faults is not None:
            self.faults.before_step(step)
            params = [p for g in self.optimizer.param_groups for p in g["params"]]
            hook = lambda: self.faults.corrupt_grads(step, params)  # noqa: E731
        self._step(images, labels, fill=fill, before_update=hook)
        self.global_step += 1
        self._tick()

    def _tick(self):
        if self.watchdog is not None:
            self.watchdog.note(f"{self.global_step} training steps queued")
            self.watchdog.tick()

    def _graph(self, k: int) -> CapturedStep | None:
        if not self.use_graph:
            return None
        if k in self._graphs:
            return self._graphs[k]
        snap = _snapshot(self.model, self.optimizer, self.scaler)
        g = CapturedStep(lambda: self._step(), warmup=2, steps_per_graph=k,
                         pre_capture=lambda: _restore(self.model, self.optimizer, self.scaler, snap))
        ctr = self.loader._ctr.clone() if self.loader._ctr is not None else None
        ok = g.capture()
        # undo the warm-up step's data consumption and parameter update
        _restore(self.model, self.optimizer, self.scaler, snap)
        if ctr is not None:
            self.loader._ctr.copy_(ctr)
        if not ok:
            self.graph_error = g.capture_error
            self.use_graph = False
            return None
        self._graphs[k] = g
        return g

    def run_epoch(self) -> None:
        self.model.train()
        sizes = self.loader.batch_sizes()
        B = self.loader.batch_size
        nfull = sum(1 for b in sizes if b == B)
        tail = [b for b in sizes if b != B]
        self.loader.start_epoch()
        done = 0
        faults = self.faults
        with trace_range("train_epoch"):
            if self.use_graph and nfull > 0:
                big = self._graph(self.spg) if nfull >= self.spg else None
                while big is not None and nfull - done >= self.spg:
                    if faults is not None and faults.pending_in(self.global_step, self.global_step + self.spg):
                        break  # run the chunk holding the fault step by step
                    big.run()
                    done += self.spg
                    self.global_step += self.spg
                    self._tick()
                if nfull - done > 0:
                    one = self._graph(1)
                    while one is not None and done < nfull:
                        if faults is not None and faults.pending_in(self.global_step, self.global_step + 1):
                            self._eager_step()
                        else:
                            one.run()
                            self.global_step += 1
                            self._tick()
                        done += 1
            while done < nfull:  # eager fallback (CPU, or capture failed)
                self._eager_step()
                done += 1
            for i, b in enumerate(tail):
                imgs, labels = self.loader.static_batch(b)
                self.loader._fill_tail(imgs, labels, nfull + i)
                self._eager_step(imgs, labels, fill=False)


@torch.no_grad()
def evaluate(model, loader: DeviceLoader, comm=None, dst: int = 0, native: bool = True):
    """Reference ``test()``: global accuracy reduced to rank ``dst`` (ddp_main.py:96-112).

    Returns (correct, size) as floats on rank ``dst`` (other ranks: their local values).
    ``native=False`` counts with torch ops (the ``--impl torch`` runs).
    """
    model.eval()
    dev = loader.device
    counters = torch.zeros(2, dtype=torch.float32, device=dev)
    native = native and dev.type == "cuda"
    if native:
        from .ops.head import accuracy_
    for images, labels in loader:
        out = model(images)
        if native:
            accuracy_(out, labels, counters)
        else:
            counters[0] += images.shape[0]
            counters[1] += (out.argmax(1) == labels).float().sum()
    if comm is not None and comm.active:
        comm.reduce_(counters, dst, "sum")
    size, correct = counters.tolist()
    return correct, size


@contextlib.contextmanager
def maybe_profile(enabled: bool, path: str):
    if not enabled:
        yield
        return
    from torch.profiler import ProfilerActivity, profile

    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    with profile(activities=acts) as prof:
        yield
    prof.export_chrome_trace(path)
