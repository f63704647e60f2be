"""SGD on the multi-tensor HIP kernel (one launch per <= 36 tensors).

Same hyper-parameters and update rule as ``torch.optim.SGD``
(torch/optim/sgd.py:29-42, foreach path :471), plus ``found_inf`` so that
``GradScaler.step`` can predicate the update on device (no host sync).

reference: /root/reference/origin_main.py:87, ddp_main.py:125 —
``torch.optim.SGD(model.parameters(), 1e-4)``.
"""
from __future__ import annotations

import os

import torch
from torch.optim import Optimizer

from .._ext import load as _load_ext


def _undecorated(name):
    """``torch.optim.Optimizer.<name>`` without its ``torch._disable_dynamo`` wrapper.

    The wrapper imports ``torch._dynamo`` on first use (~1.2 s, measured: the largest
    single cost of a 3-epoch CLI run); this framework never traces an optimizer, so the
    plain function is called.
    """
    fn = getattr(Optimizer, name)
    return getattr(fn, "__wrapped__", fn)


# the plain step on the fused launch (slab sums and the deferred DDP average inside it);
# DPA_PLAIN_FUSED=0: the multi-tensor SGD launch after separate reductions (A/B runs)
_PLAIN_FUSED = os.environ.get("DPA_PLAIN_FUSED", "1") != "0"


class SGD(Optimizer):
    supports_device_found_inf = True
    # step() without a GradScaler runs the fused launch when _fuse_kind() is "small", so
    # the engine may hand it the deferred slab / DDP average (engine.TrainLoop)
    plain_fused = _PLAIN_FUSED

    add_param_group = _undecorated("add_param_group")
    zero_grad = _undecorated("zero_grad")
    state_dict = _undecorated("state_dict")
    load_state_dict = _undecorated("load_state_dict")

    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, *, maximize: bool = False):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if momentum < 0.0:
            raise ValueError(f"Invalid momentum value: {momentum}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, maximize=maximize)
        super().__init__(params, defaults)
        # grid-barrier state of the fused AMP step, zeroed here, outside any graph capture:
        # created lazily inside a capture, its zero-fill became a graph node that re-ran on
        # every replay (profiles/r4final_convnet_steady.txt)
        ps = [p for g in self.param_groups for p in g["params"]]
        if ps and all(p.is_cuda for p in ps) and len({p.device for p in ps}) == 1:
            self._amp_sync = torch.zeros(4, dtype=torch.int64, device=ps[0].device)
            self._amp_sync_large = torch.zeros(4, dtype=torch.int64, device=ps[0].device)
            # the deferred-wgrad1 launch's barrier state (convnet_amp_step): generation,
            # 2 parities x 8 arrival words 64 B apart, error word; and the conv1 arrival counter
            self._amp_sync_cas = (torch.zeros(1 + 2 * 8 * 8 + 1, dtype=torch.int64, device=ps[0].device),
                                  torch.zeros(1, dtype=torch.int32, device=ps[0].device))

    def defer_slab(self, slab: torch.Tensor, out: torch.Tensor) -> None:
        """A gradient region ``out`` that is still the partial rows ``slab`` [rows][out.numel()]
        of its producer (the ConvNet's conv1 weight gradient, ops/convnet_fused.py): the next
        fused AMP step sums the columns inside its own launch (csrc/kernels/optim.hip
        SlabSrc); any other gradient reader flushes first (``_flush_deferred``)."""
        self.flush_slab()
        self._pending_slab = (slab, out)

    def defer_wgrad1(self, w: dict) -> None:
        """The ConvNet's conv1 weight gradient -- with BN1's and conv2's gradient column sums
        -- left undone by the backward (ops/convnet_fused.py): the next fused AMP step
        computes it inside its own launch (csrc/kernels/convnet_fused.hip convnet_amp_step),
        so the update still happens in ``scaler.step()``; any other gradient reader
        flushes first (``flush_slab``)."""
        self.flush_slab()
        self._pending_wgrad1 = w

    def grad_chk(self, n: int, device) -> torch.Tensor | None:
        """The int32 words of the ConvNet's producer-side gradient check (ops/convnet_fused.py:
        the head launch clears them, the backward launches set them; no zero-fill).  Created
        outside a graph capture only; None inside one when they do not exist yet."""
        t = self.__dict__.get("_grad_chk")
        if t is None or t.numel() != n or t.device != device:
            if device.type == "cuda" and torch.cuda.is_current_stream_capturing():
                return None
            t = self._grad_chk = torch.empty(n, dtype=torch.int32, device=device)
        return t

    def set_prechecked(self, chk: torch.Tensor, scale: torch.Tensor, out: torch.Tensor) -> None:
        """The gradients in ``out`` (one buffer holding every parameter's) were checked by their
        producers against ``scale``: the next fused AMP step may read ``chk`` instead of agreeing
        on found_inf at a grid barrier.  Any other gradient reader drops it (flush_slab)."""
        self._prechecked = (chk, scale, out.data_ptr(), out.data_ptr() + out.numel() * out.element_size())

    def clear_prechecked(self) -> None:
        self.__dict__.pop("_prechecked", None)

    def flush_slab(self) -> None:
        self.__dict__.pop("_prechecked", None)  # .grad may be read or changed from here on
        w = self.__dict__.pop("_pending_wgrad1", None)
        if w is not None:  # the launches the deferral saved
            C = _load_ext()
            out0 = w["out0"]  # [dbeta1 | dgamma1]
            C.convnet.conv1_wgrad_slab2(w["x"], w["y1"], w["dp1"], w["idx1"], w["fstats1"], w["gsum1"], w["lsum1"],
                                        w["g1"], w["e1"], out0.narrow(0, 16, 16), out0.narrow(0, 0, 16), w["wslab1"],
                                        w["wslab2"], w["out2"], w["xc1"], None)
            C.convblock.slab_reduce(w["wslab1"], w["out1"].numel(), w["out1"])
        ps = self.__dict__.pop("_pending_slab", None)
        if ps is not None:
            _load_ext().convblock.slab_reduce(ps[0], ps[1].numel(), ps[1])

    def _flush_deferred(self):
        """Average gradients a DDP reducer left to this optimizer (DDP.defer_grad_sync_to)
        and sum a deferred gradient slab (defer_slab)."""
        self.flush_slab()
        d = getattr(self, "_deferred_ddp", None)
        if d is not None:
            d[0].flush_deferred()

    @torch.no_grad()
    def step(self, closure=None, found_inf: torch.Tensor | None = None):
        if closure is None and found_inf is None and _PLAIN_FUSED and self._fuse_kind() == "small":
            self._fused_plain_step()
            return None
        self._flush_deferred()
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group, params, grads, bufs, first in self._collect():
            if not params:
                continue
            native = params[0].is_cuda and all(
                p.dtype == torch.float32 and p.is_contiguous() and g.dtype == torch.float32 and g.is_contiguous()
                for p, g in zip(params, grads))
            if native:
                _load_ext().optim.sgd_step(params, grads, bufs, group["lr"], group["momentum"], group["dampening"],
                                           group["weight_decay"], group["nesterov"], group["maximize"], first,
                                           found_inf, None)
            else:
                if found_inf is not None and bool(found_inf.item()):
                    continue
                self._torch_step(group, params, grads, bufs, first)
        return loss

    # ------------------------------------------------------------------ AMP
    FUSED_AMP_MAX_NUMEL = 1 << 19  # csrc/kernels/optim.hip FUSED_MAX

    def _collect(self):
        """Per group: params with a grad, their grads and momentum buffers, and one "first"
        flag per tensor (its buffer was just created: torch's ``buf = d`` step).

        Buffers start at zero, so with dampening 0 the first step's ``momentum*0 + d``
        IS ``d``: no flag is passed then, which also keeps a device-skipped first step
        (found_inf) exact -- the buffer simply stays zero.  With dampening != 0 the flags
        are per tensor; a first step skipped on the device consumes them (documented gap).
        """
        out = []
        for group in self.param_groups:
            params, grads, bufs, first = [], [], [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                params.append(p)
                grads.append(p.grad)
                if group["momentum"] != 0:
                    st = self.state[p]
                    new = st.get("momentum_buffer") is None
                    if new:
                        st["momentum_buffer"] = torch.zeros_like(p)
                    bufs.append(st["momentum_buffer"])
                    first.append(int(new))
            if group["dampening"] == 0 or not any(first):
                first = []
            out.append((group, params, grads, bufs, first))
        return out

    def _fuse_kind(self) -> str | None:
        """"small": one launch of <= 128 co-resident workgroups holding every value in
        registers (<= 2^19 floats, <= 36 tensors: the ConvNet); "large": the grid-stride
        two-phase launch with a device tensor table (any size, <= 512 tensors: ResNet-50);
        None: the multi-tensor unscale / SGD / update launches."""
        if len(self.param_groups) != 1:
            return None
        ps = [p for p in self.param_groups[0]["params"] if p.grad is not None]
        if not ps:
            return None

        def aligned(t):  # the kernels move float4 granules
            return t is None or t.data_ptr() % 16 == 0

        if not all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad.dtype == torch.float32
                   and p.grad.is_contiguous() and aligned(p) and aligned(p.grad)
                   and aligned(self.state.get(p, {}).get("momentum_buffer")) for p in ps):
            return None
        O = _load_ext().optim
        # the kernel rounds every tensor up to whole float4 granules (csrc/kernels/optim.hip)
        if (len(ps) <= O.MAXT and sum((p.numel() + 3) // 4 * 4 for p in ps) <= self.FUSED_AMP_MAX_NUMEL
                and O.amp_sgd_resident()):
            return "small"
        if len(ps) <= O.LARGE_MAXT and O.amp_sgd_large_resident():
            return "large"
        return None

    def small_fusable(self) -> bool:
        """The "small" fused step will apply once the gradients exist (predicted from the
        parameters: their gradients are then fp32 views of one aligned buffer)."""
        if len(self.param_groups) != 1:
            return False
        ps = self.param_groups[0]["params"]
        if not ps or not all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.data_ptr() % 16 == 0
                             for p in ps):
            return False
        if self.param_groups[0]["momentum"] != 0:
            return False  # buffers may not exist yet (first step): keep the plain path
        O = _load_ext().optim
        return (len(ps) <= O.MAXT and sum((p.numel() + 3) // 4 * 4 for p in ps) <= self.FUSED_AMP_MAX_NUMEL
                and O.amp_sgd_resident())

    def can_fuse_amp(self) -> bool:
        """Unscale + inf-check + SGD + scale update as one launch (see _fuse_kind)."""
        return self._fuse_kind() is not None

    def _large_table(self, params, grads, bufs, first):
        """Device tensor table of the large fused step, cached per set of pointers (DDP
        bucket-view grads and the optimizer state keep them fixed; freshly allocated
        grads may not).  Any table looked up during graph capture -- built then, or an
        eager warm-up's table reused from the cache -- stays referenced for the life of
        the optimizer (the graph reads it on every replay).  The key carries every
        tensor's size too: memory reused at the same address for a different size must
        not hit a stale table."""
        key = (tuple((p.data_ptr(), p.numel()) for p in params), tuple((g.data_ptr(), g.numel()) for g in grads),
               tuple((b.data_ptr(), b.numel()) for b in bufs), tuple(first))
        cache = self.__dict__.setdefault("_amp_tables", {})
        t = cache.get(key)
        if t is None:
            t = _load_ext().optim.amp_sgd_table(params, grads, bufs, first)
            if len(cache) >= 8:  # eager tables: the allocator's stream order makes freeing safe
                cache.pop(next(iter(cache)))
            cache[key] = t
        if torch.cuda.is_current_stream_capturing():
            pinned = self.__dict__.setdefault("_amp_tables_pinned", [])
            if not any(x is t for x in pinned):
                pinned.append(t)
        return t

    @torch.no_grad()
    def fused_amp_step(self, scale, tracker, found_inf, growth, backoff, interval):
        (group, params, grads, bufs, first), = self._collect()
        kind = self._fuse_kind()
        name = "_amp_sync" if kind == "small" else "_amp_sync_large"
        sync = getattr(self, name, None)
        if sync is None or sync.device != params[0].device:
            # grid-barrier state of the fused kernel (allocated before any graph capture:
            # the first step runs eagerly)
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("SGD: the fused AMP step's barrier state must exist before graph capture "
                                   "(run one eager step first)")
            sync = torch.zeros(4, dtype=torch.int64, device=params[0].device)
            setattr(self, name, sync)
        O = _load_ext().optim
        pc = self.__dict__.pop("_prechecked", None)
        w1 = self.__dict__.get("_pending_wgrad1")
        if w1 is not None and kind != "small":
            self.flush_slab()
            w1 = None
        if kind == "large":
            self._flush_deferred()
            O.amp_sgd_large(self._large_table(params, grads, bufs, first), group["lr"], group["momentum"],
                            group["dampening"], group["weight_decay"], group["nesterov"], group["maximize"],
                            scale, tracker, found_inf, growth, backoff, interval, sync)
            return
        # gradients a DDP reducer deferred to this step are averaged inside the kernel
        d = getattr(self, "_deferred_ddp", None)
        xc = d[1] if d is not None and d[0].deferred_pending() else None
        if w1 is not None:
            # conv1's weight gradient + the slab sums + this step in one launch
            del self._pending_wgrad1
            cas = getattr(self, "_amp_sync_cas", None)
            if cas is None or cas[0].device != params[0].device:
                # allocated in __init__; created here only for parameters moved since, and
                # never inside a capture (its zero-fill would become a node re-run, and the
                # barrier generation reset, on every replay)
                if torch.cuda.is_current_stream_capturing():
                    raise RuntimeError("SGD: the fused AMP step's barrier state must exist before graph capture "
                                       "(run one eager step first)")
                cas = self._amp_sync_cas = (torch.zeros(1 + 2 * 8 * 8 + 1, dtype=torch.int64, device=params[0].device),
                                            torch.zeros(1, dtype=torch.int32, device=params[0].device))
            _load_ext().convnet.convnet_amp_step(
                params, grads, bufs, group["lr"], group["momentum"], group["dampening"], group["weight_decay"],
                group["nesterov"], group["maximize"], first, scale, tracker, found_inf, growth, backoff, interval,
                cas[0], xc, w1["x"], w1["y1"], w1["dp1"], w1["idx1"], w1["fstats1"], w1["gsum1"], w1["g1"], w1["e1"],
                w1["wslab1"], cas[1], w1["out1"], w1["bn1"], w1["out0"], w1["wslab2"], w1["out2"])
            if xc is not None:
                d[0].consume_deferred()
            return
        # summed inside the launch (SlabSrc), and exchanged there with the other gradients
        # when the DDP average is fused in too (xc)
        ps = self.__dict__.pop("_pending_slab", None)
        # producer-checked gradients (ops/convnet_fused.py): every gradient lies in the checked
        # buffer and was checked against this scale -> no grid barrier in the launch.  Under a
        # deferring DDP reducer only with the average in this launch (xc: a flagged rank
        # poisons its pushed values, csrc/kernels/amp_step.h), never after a reducer all-reduce
        prechk = None
        if (pc is not None and ps is not None and pc[1] is scale and (xc is not None or d is None)
                and all(pc[2] <= g.data_ptr() < pc[3] for g in grads)):
            prechk = pc[0]
        O.amp_sgd_fused(params, grads, bufs, group["lr"], group["momentum"], group["dampening"],
                        group["weight_decay"], group["nesterov"], group["maximize"], first,
                        scale, tracker, found_inf, growth, backoff, interval, sync, xc,
                        ps[0] if ps is not None else None, ps[1] if ps is not None else None, prechk)
        if xc is not None:
            d[0].consume_deferred()

    def _fused_plain_step(self):
        """torch.optim.SGD's update as one launch of the fused kernel without a scale
        (csrc/kernels/amp_step.h amp_sgd_body, plain mode): a deferred conv1 slab is summed
        and a deferred DDP average exchanged inside it, as in the AMP step."""
        (group, params, grads, bufs, first), = self._collect()
        if "_pending_wgrad1" in self.__dict__:
            self.flush_slab()  # the AMP-only deferral (convnet_amp_step): its launches first
        sync = getattr(self, "_amp_sync", None)
        if sync is None or sync.device != params[0].device:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("SGD: the fused step's state must exist before graph capture "
                                   "(run one eager step first)")
            sync = self._amp_sync = torch.zeros(4, dtype=torch.int64, device=params[0].device)
        d = getattr(self, "_deferred_ddp", None)
        xc = d[1] if d is not None and d[0].deferred_pending() else None
        ps = self.__dict__.pop("_pending_slab", None)
        _load_ext().optim.amp_sgd_fused(params, grads, bufs, group["lr"], group["momentum"], group["dampening"],
                                        group["weight_decay"], group["nesterov"], group["maximize"], first,
                                        None, None, None, 1.0, 1.0, 1, sync, xc,
                                        ps[0] if ps is not None else None, ps[1] if ps is not None else None)
        if xc is not None:
            d[0].consume_deferred()

    @staticmethod
    def _torch_step(group, params, grads, bufs, first):
        lr, mom, damp, wd = group["lr"], group["momentum"], group["dampening"], group["weight_decay"]
        for i, (p, g) in enumerate(zip(params, grads)):
            d = -g if group["maximize"] else g
            if wd != 0:
                d = d.add(p, alpha=wd)
            if mom != 0:
                b = bufs[i]
                if first and first[i]:
                    b.copy_(d)
                else:
                    b.mul_(mom).add_(d, alpha=1 - damp)
                d = d.add(b, alpha=mom) if group["nesterov"] else b
            p.add_(d, alpha=-lr)
