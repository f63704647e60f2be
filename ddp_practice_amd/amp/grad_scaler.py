"""Dynamic loss scaling with all state resident on the device.

Semantics follow ``torch.amp.GradScaler`` (torch/amp/grad_scaler.py:123-129
defaults; scale :190-222; unscale_ :235-286; step :348-357; update :500-537;
state_dict :607-632), with one structural difference: ``step`` never calls
``found_inf.item()``.  When the optimizer is this package's fused SGD the
inf-check result is consumed on the device (the SGD kernel is predicated on
``found_inf``), so a whole training step — forward, backward, all-reduce,
unscale, step, scale update — can be captured in one hipGraph.  For any other
optimizer the host-synchronising fallback of the reference is used.

reference: /root/reference/ddp_main.py:10,126 (``GradScaler()``), :91-93.
"""
from __future__ import annotations

import weakref
from typing import Any

import torch

from .._ext import load as _load_ext

_ACTIVE = None  # weakref to the GradScaler whose scale native losses pre-apply


def active_scale(device: torch.device):
    """Scale tensor of the active GradScaler on ``device`` (or None).

    Native losses (ops/head.py cross_entropy) use it to write the gradient of
    the *scaled* loss in their forward kernel; ``GradScaler.scale`` then hands
    out that pre-scaled loss and its fast backward needs neither the
    ``loss * scale`` multiply nor the loss-backward launch.
    """
    sc = _ACTIVE() if _ACTIVE is not None else None
    if sc is None or not sc._enabled or device.type != "cuda":
        return None
    if sc._scale is None:
        # a fresh scaler: create its scale now, so the very first step takes the same
        # (pre-scaled) loss path as every later one -- eager and graph-captured training
        # then run identical kernels from step 0 on
        sc._lazy_init(device)
    return sc._scale if sc._scale.device == device else None


class _ScaledLossFn(torch.autograd.Function):
    """scale * loss whose value the loss kernel already produced (no launch)."""

    @staticmethod
    def forward(ctx, loss, scale, ce_node):
        ctx.save_for_backward(scale)
        out = ce_node.scaled  # a view of the loss kernel's output buffer: no launch
        # the loss node must not keep this output alive: it becomes the output of THIS node,
        # whose edge leads back to the loss node -- a reference cycle that kept every
        # step's autograd graph (AccumulateGrad nodes included) alive until the cyclic GC
        # ran; graph capture after eager steps then synchronised with their stream
        ce_node.scaled = None
        return out

    @staticmethod
    def backward(ctx, g):
        (scale,) = ctx.saved_tensors
        return g * scale.view(()).to(g.dtype), None, None


def _native_ok(t: torch.Tensor) -> bool:
    return t.is_cuda



def _seeded_backward(t: torch.Tensor, seed: torch.Tensor, retain_graph, inputs) -> None:
    """``torch.autograd.backward(t, grad_tensors=seed)`` for a 0-d ``t`` and a 0-d floating
    seed on its device, straight into the autograd engine (which casts the seed to ``t``'s
    dtype, as torch's own path does).

    torch's ``_make_grads`` only validates the seed's shape here, and doing so imports
    ``torch.fx.experimental.symbolic_shapes`` (sympy) on first use: 1.35 s of the first
    training step on a fresh box (measured with cProfile, ``scripts/prof_cli_ddp.sh``).
    """
    run = getattr(torch.autograd.graph, "_engine_run_backward", None)
    if (run is None or seed.shape != t.shape or seed.device != t.device or not seed.is_floating_point()
            or not t.is_floating_point()):
        torch.autograd.backward(t, grad_tensors=seed, retain_graph=retain_graph, inputs=inputs)
        return
    if inputs is None:
        inputs_t = ()
    elif isinstance(inputs, (torch.Tensor, torch.autograd.graph.GradientEdge)):
        inputs_t = (inputs,)
    else:
        inputs_t = tuple(inputs)
        if not inputs_t:
            raise RuntimeError("`inputs` argument to `backward()` cannot be empty.")
    run((t,), (seed,), bool(retain_graph), False, inputs_t, allow_unreachable=True, accumulate_grad=True)

class GradScaler:
    def __init__(self, device: str = "cuda", init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000, enabled: bool = True,
                 fuse_step: bool = True):
        if growth_factor <= 1.0:
            raise ValueError("growth_factor should be > 1")
        if not (0.0 < backoff_factor < 1.0):
            raise ValueError("backoff_factor should be < 1")
        self._device = device if (device != "cuda" or torch.cuda.is_available()) else "cpu"
        self._enabled = enabled
        self._init_scale = float(init_scale)
        self._growth_factor = float(growth_factor)
        self._backoff_factor = float(backoff_factor)
        self._growth_interval = int(growth_interval)
        self._scale: torch.Tensor | None = None
        self._growth_tracker: torch.Tensor | None = None
        self._found_inf: torch.Tensor | None = None
        self._per_opt: dict[int, dict[str, Any]] = {}
        self._armed = True  # device found_inf is known to be 0
        # fused single-launch step: enabled once an iteration with exactly one
        # optimizer has been seen (the fused kernel also performs update())
        self._fuse_step = fuse_step
        self._single_opt_iters = 0
        self._fused_done = False
        if enabled and str(self._device).startswith("cuda"):
            global _ACTIVE
            _ACTIVE = weakref.ref(self)  # the newest scaler is the one native losses pre-scale for

    # ------------------------------------------------------------------ state
    def _lazy_init(self, dev: torch.device):
        global _ACTIVE
        if self._enabled and dev.type == "cuda":
            _ACTIVE = weakref.ref(self)
        if self._scale is None:
            self._scale = torch.full((1,), self._init_scale, dtype=torch.float32, device=dev)
            self._growth_tracker = torch.full((1,), getattr(self, "_pending_tracker", 0), dtype=torch.int32,
                                              device=dev)
            self._found_inf = torch.zeros((1,), dtype=torch.float32, device=dev)

    def is_enabled(self) -> bool:
        return self._enabled

    def get_scale(self) -> float:
        if not self._enabled:
            return 1.0
        return self._init_scale if self._scale is None else float(self._scale.item())

    @property
    def scale_tensor(self) -> torch.Tensor:
        return self._scale

    @property
    def found_inf(self) -> torch.Tensor:
        return self._found_inf

    # ------------------------------------------------------------------ API
    def scale(self, outputs):
        if not self._enabled:
            return outputs
        if isinstance(outputs, torch.Tensor):
            self._lazy_init(outputs.device)
            # 0-d scale: a 0-d loss stays 0-d, so backward needs no sum-to-shape reduction
            s0 = self._scale.to(outputs.device, non_blocking=True).view(())
            ce = getattr(outputs, "_dpa_ce", None)
            # the pre-scaled value is handed out once (see _ScaledLossFn); a second scale() of
            # the same loss (logging, a retry) takes the generic multiply below
            if (ce is not None and ce[1] is self._scale and getattr(ce[0], "scaled", None) is not None
                    and outputs.requires_grad and outputs.dim() == 0):
                # native CE loss: its kernel already wrote loss*scale and d(scale*loss)/dlogits
                node = ce[0]
                scaled = _ScaledLossFn.apply(outputs, self._scale, node)
                base = outputs
                # weak: the closure is stored on `scaled` itself; a strong reference would be a
                # reference cycle keeping the step's whole autograd graph alive until the cyclic
                # GC runs (a later hipGraph capture then syncs with the old nodes' stream)
                scaled_ref = weakref.ref(scaled)

                def _backward_ce(gradient=None, retain_graph=None, create_graph=False, inputs=None):
                    if gradient is None and not create_graph:
                        node.token.seeded = True
                        try:
                            _seeded_backward(base, s0, retain_graph, inputs)
                        finally:
                            node.token.seeded = False
                    else:
                        torch.Tensor.backward(scaled_ref(), gradient, retain_graph, create_graph, inputs)

                scaled.backward = _backward_ce
                return scaled
            scaled = outputs * s0
            if outputs.requires_grad and outputs.dim() == 0 and outputs.is_cuda:
                # d(scale*loss)/dθ = scale * dloss/dθ: seed the loss's own backward
                # with the scale tensor instead of a ones() fill + MulBackward kernel
                # pair (2 fewer launches per step); any other use of `scaled`
                # (extra terms, retain/create_graph, explicit gradient) goes
                # through normal autograd.
                base = outputs
                seed = s0 if base.dtype == torch.float32 else s0.to(base.dtype)
                scaled_ref = weakref.ref(scaled)  # no reference cycle (see above)

                def _backward(gradient=None, retain_graph=None, create_graph=False, inputs=None):
                    if gradient is None and not create_graph:
                        _seeded_backward(base, seed, retain_graph, inputs)
                    else:
                        torch.Tensor.backward(scaled_ref(), gradient, retain_graph, create_graph, inputs)

                scaled.backward = _backward
            return scaled
        if isinstance(outputs, (list, tuple)):
            return type(outputs)(self.scale(o) for o in outputs)
        raise ValueError("outputs must be a Tensor or an iterable of Tensors")

    def _grads(self, optimizer):
        gs = []
        for group in optimizer.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise NotImplementedError("sparse grads are not supported")
                gs.append(p.grad)
        return gs

    def unscale_(self, optimizer):
        if not self._enabled:
            return
        st = self._per_opt.setdefault(id(optimizer), {"stage": "ready"})
        if st["stage"] == "unscaled":
            raise RuntimeError("unscale_() has already been called on this optimizer since the last update().")
        if st["stage"] == "stepped":
            raise RuntimeError("unscale_() is being called after step().")
        flush = getattr(optimizer, "_flush_deferred", None)  # DDP.defer_grad_sync_to: average first
        if flush is not None:
            flush()
        grads = self._grads(optimizer)
        if self._scale is None:
            self._lazy_init(grads[0].device if grads else torch.device(self._device))
        native = grads and _native_ok(grads[0]) and all(g.dtype == torch.float32 and g.is_contiguous()
                                                           for g in grads)
        if not (native and self._armed):
            self._found_inf.zero_()
        self._armed = False
        if native:
            _load_ext().optim.unscale_check(grads, self._scale, self._found_inf)
        else:
            inv = self._scale.double().reciprocal().float()
            for g in grads:
                self._found_inf.copy_(torch.maximum(self._found_inf, (~torch.isfinite(g)).any().float().reshape(1)))
                g.mul_(inv.to(g.dtype))
        st["stage"] = "unscaled"

    def step(self, optimizer, *args, **kwargs):
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        if "closure" in kwargs:
            raise RuntimeError("Closure use is not currently supported if GradScaler is enabled.")
        st = self._per_opt.setdefault(id(optimizer), {"stage": "ready"})
        if st["stage"] == "stepped":
            raise RuntimeError("step() has already been called since the last update().")
        if self._fused_done:
            raise RuntimeError("GradScaler: a fused AMP step already updated the scale in this iteration; "
                               "use GradScaler(fuse_step=False) with several optimizers")
        if (st["stage"] == "ready" and self._fuse_step and self._single_opt_iters >= 1 and self._scale is not None
                and self._scale.is_cuda and getattr(optimizer, "can_fuse_amp", lambda: False)()):
            # unscale + inf-check + SGD + scale update in one launch (update() becomes bookkeeping)
            optimizer.fused_amp_step(self._scale, self._growth_tracker, self._found_inf, self._growth_factor,
                                     self._backoff_factor, self._growth_interval)
            self._fused_done = True
            st["stage"] = "stepped"
            return None
        if st["stage"] == "ready":
            self.unscale_(optimizer)
        ret = None
        if getattr(optimizer, "supports_device_found_inf", False):
            # fused path: the optimizer kernel reads found_inf on device (no host sync)
            ret = optimizer.step(*args, found_inf=self._found_inf, **kwargs)
        else:
            if not bool(self._found_inf.item()):
                ret = optimizer.step(*args, **kwargs)
        st["stage"] = "stepped"
        return ret

    def update(self, new_scale=None):
        if not self._enabled:
            return
        if self._scale is None:
            return
        self._single_opt_iters = self._single_opt_iters + 1 if len(self._per_opt) == 1 else 0
        if self._fused_done:
            # the fused step kernel already updated scale / tracker and re-armed found_inf
            self._fused_done = False
            self._armed = True
            if new_scale is not None:
                self._scale.fill_(new_scale) if isinstance(new_scale, float) else self._scale.copy_(new_scale)
            self._per_opt = {}
            return
        if new_scale is not None:
            if isinstance(new_scale, float):
                self._scale.fill_(new_scale)
            else:
                self._scale.copy_(new_scale)
        else:
            if self._scale.is_cuda:
                # also re-arms found_inf to 0 on device (no separate fill launch)
                _load_ext().optim.update_scale(self._scale, self._growth_tracker, self._found_inf,
                                               self._growth_factor, self._backoff_factor, self._growth_interval)
                self._armed = True
            else:
                torch._amp_update_scale_(self._scale, self._growth_tracker, self._found_inf,
                                         self._growth_factor, self._backoff_factor, self._growth_interval)
        self._per_opt = {}

    # ------------------------------------------------------------ checkpoint
    def get_growth_factor(self):
        return self._growth_factor

    def get_backoff_factor(self):
        return self._backoff_factor

    def get_growth_interval(self):
        return self._growth_interval

    def _get_growth_tracker(self) -> int:
        if self._growth_tracker is None:
            return 0
        return int(self._growth_tracker.item())

    def state_dict(self) -> dict[str, Any]:
        """Same keys/types as torch.amp.GradScaler.state_dict()."""
        if not self._enabled:
            return {}
        return {
            "scale": self.get_scale(),
            "growth_factor": self._growth_factor,
            "backoff_factor": self._backoff_factor,
            "growth_interval": self._growth_interval,
            "_growth_tracker": self._get_growth_tracker(),
        }

    def load_state_dict(self, state_dict: dict[str, Any]):
        if not self._enabled:
            return
        if len(state_dict) == 0:
            raise RuntimeError("The source state dict is empty, possibly because it was saved from a disabled "
                               "instance of GradScaler.")
        self._init_scale = float(state_dict["scale"])
        if self._scale is not None:
            self._scale.fill_(state_dict["scale"])
        self._growth_factor = float(state_dict["growth_factor"])
        self._backoff_factor = float(state_dict["backoff_factor"])
        self._growth_interval = int(state_dict["growth_interval"])
        if self._growth_tracker is not None:
            self._growth_tracker.fill_(int(state_dict["_growth_tracker"]))
        else:
            self._pending_tracker = int(state_dict["_growth_tracker"])
