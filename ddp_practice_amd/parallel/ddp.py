"""DistributedDataParallel over the native communicator + C++ reducer.

Contract of torch.nn.parallel.DistributedDataParallel as the reference uses it
(/root/reference/ddp_main.py:121-123: ``DDP(model, device_ids=[local_rank])``):
  * construction: parameter-shape check across ranks, then rank 0's
    parameters and buffers are broadcast (torch/nn/parallel/distributed.py:825,860-872);
  * every training forward: buffers broadcast from rank 0 when
    ``broadcast_buffers`` (distributed.py:1521-1558) — skipped when every buffer
    belongs to a SyncBatchNorm, whose running stats are computed from globally
    reduced statistics and are therefore already identical on all ranks;
  * backward: gradients averaged over ranks by bucketed all-reduce overlapped
    with the remaining backward (C++ Reducer, csrc/ddp/reducer.cpp);
  * ``state_dict()`` keys carry the ``module.`` prefix; ``no_sync()``;
    ``find_unused_parameters``.

Bucket sizing for MI355X: RCCL over xGMI is latency-bound below ~1 MB and
per-link-bandwidth bound above (7 x ~153 GB/s links per GPU, ring algorithms
use one link per direction).  Fewer, larger buckets amortise the ~10-30 us
per-collective latency; the first bucket stays small (1 MiB) so the
all-reduce of the last layers' gradients starts while early layers are still
in backward.  Default cap 32 MiB (HBM is 288 GB, memory is not the limit).
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.nn as nn

from .._ext import load as _load_ext
from . import comm as _comm
from .sync_bn import SyncBatchNorm

DEFAULT_FIRST_BUCKET_MB = 1.0
DEFAULT_BUCKET_CAP_MB = 32.0


def compute_bucket_assignment(params, cap_bytes: float, first_bytes: float, order=None) -> list[list[int]]:
    """Greedy bucketing in `order` (default: reverse parameter order), per dtype/device.

    Same algorithm as torch's _compute_bucket_assignment_by_size: a bucket closes
    once its byte size reaches the current limit; limits are [first, cap, cap, ...].
    """
    if order is None:
        order = list(range(len(params) - 1, -1, -1))
    open_b: dict = {}
    limits_idx: dict = {}
    out: list[list[int]] = []
    limits = [first_bytes, cap_bytes]
    for i in order:
        p = params[i]
        key = (p.dtype, p.device)
        b = open_b.setdefault(key, [[], 0])
        b[0].append(i)
        b[1] += p.numel() * p.element_size()
        li = limits_idx.get(key, 0)
        if b[1] >= limits[min(li, 1)]:
            out.append(b[0])
            open_b[key] = [[], 0]
            limits_idx[key] = li + 1
    for b in open_b.values():
        if b[0]:
            out.append(b[0])
    return out


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None, dim: int = 0,
                 broadcast_buffers: bool = True, process_group=None, bucket_cap_mb: float | None = None,
                 find_unused_parameters: bool = False, check_reduction: bool = False,
                 gradient_as_bucket_view: bool = False, static_graph: bool = False,
                 first_bucket_mb: float | None = None):
        super().__init__()
        self.module = module
        # the wrapped model's gradients are read by the reducer's hooks mid-backward: no
        # end-of-backward deferral of their values (ops/conv_igemm.WgradBatch)
        module._dpa_ddp_wrapped = True
        self.device_ids = device_ids
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.static_graph = static_graph
        # False (torch's default): after the all-reduce the averaged values are copied back into
        # the gradient tensors autograd produced; True: param.grad become views of the buckets
        self.gradient_as_bucket_view = gradient_as_bucket_view
        self.comm = process_group if isinstance(process_group, _comm.Communicator) else _comm.default_comm()
        self.bucket_cap_bytes = (bucket_cap_mb if bucket_cap_mb is not None else DEFAULT_BUCKET_CAP_MB) * 2 ** 20
        self.first_bucket_bytes = (first_bucket_mb if first_bucket_mb is not None
                                   else DEFAULT_FIRST_BUCKET_MB) * 2 ** 20
        self._params = [p for p in module.parameters() if p.requires_grad]
        if len({id(p) for p in self._params}) != len(self._params):
            raise RuntimeError("DDP does not support shared parameters listed twice")
        self._sync_enabled = True
        self._iteration = 0
        self._rebuilt = False
        self.require_forward_param_sync = True
        self._verify_param_shapes()
        self._sync_module_states()
        self._buffers_need_sync = broadcast_buffers and any(
            not isinstance(self._owner_of_buffer(name), (SyncBatchNorm, nn.SyncBatchNorm))
            for name, _ in module.named_buffers())
        self.reducer = None
        if self.comm.active and self._params:
            buckets = compute_bucket_assignment(self._params, self.bucket_cap_bytes, self.first_bucket_bytes)
            self.reducer = _load_ext().ddp.Reducer(self._params, buckets, self.comm.native, find_unused_parameters)
            if not gradient_as_bucket_view:
                self.reducer.set_grad_as_view(False)

    # ------------------------------------------------------------- init sync
    def _owner_of_buffer(self, name: str):
        mod = self.module
        parts = name.split(".")
        for p in parts[:-1]:
            mod = getattr(mod, p)
        return mod

    _DTYPE_CODES = {torch.float32: 1, torch.float16: 2, torch.bfloat16: 3, torch.float64: 4}
    _MAX_DIMS = 8

    def _param_table(self) -> torch.Tensor:
        """One int64 row per parameter: [ndim, dtype, dim0 .. dim7 (-1 padded)]."""
        rows = []
        for p in self._params:
            if p.dim() > self._MAX_DIMS:
                raise RuntimeError(f"DDP: parameters of more than {self._MAX_DIMS} dims are not supported")
            dims = list(p.shape) + [-1] * (self._MAX_DIMS - p.dim())
            rows.append([p.dim(), self._DTYPE_CODES.get(p.dtype, 99)] + dims)
        return torch.tensor(rows, dtype=torch.int64).reshape(len(rows), 2 + self._MAX_DIMS)

    def _verify_param_shapes(self):
        """Exact parameter count, shapes and dtypes on every rank (torch's
        _verify_param_shape_across_processes, torch/distributed/utils.py:281): the count
        first (every rank must gather the same number of rows), then the whole table,
        compared row by row with rank 0's."""
        if self.comm.world_size == 1:
            return
        W, dev = self.comm.world_size, self.comm.device
        n = torch.tensor([len(self._params)], dtype=torch.int64, device=dev)
        counts = torch.empty(W, dtype=torch.int64, device=dev)
        self.comm.all_gather_into_tensor(counts, n)
        counts = counts.cpu().tolist()
        if len(set(counts)) != 1:
            raise RuntimeError(f"DDP expects the same model on every rank, but the ranks have {counts} "
                               f"parameters (rank {self.comm.rank} has {len(self._params)})")
        if not self._params:
            return
        mine = self._param_table()
        every = torch.empty((W,) + tuple(mine.shape), dtype=torch.int64, device=dev)
        self.comm.all_gather_into_tensor(every, mine.to(dev).contiguous())
        every = every.cpu()
        codes = {v: k for k, v in self._DTYPE_CODES.items()}
        for r in range(1, W):
            bad = (every[r] != every[0]).any(dim=1).nonzero().flatten().tolist()
            if bad:
                i = bad[0]

                def desc(row):
                    nd = int(row[0])
                    return f"shape {tuple(int(d) for d in row[2:2 + nd])} dtype {codes.get(int(row[1]), 'other')}"

                raise RuntimeError(f"DDP expects the same model on every rank, but parameter {i} has "
                                   f"{desc(every[r][i])} on rank {r} and {desc(every[0][i])} on rank 0")

    def _flat_broadcast(self, tensors):
        by_dtype: dict = {}
        for t in tensors:
            by_dtype.setdefault(t.dtype, []).append(t)
        for ts in by_dtype.values():
            flat = torch.cat([t.detach().reshape(-1) for t in ts])
            self.comm.broadcast_(flat, 0)
            off = 0
            with torch.no_grad():
                for t in ts:
                    n = t.numel()
                    t.copy_(flat[off:off + n].view_as(t))
                    off += n

    def _sync_module_states(self):
        if self.comm.world_size == 1:
            return
        ts = [p.data for p in self.module.parameters()] + [b for b in self.module.buffers()]
        if ts:
            self._flat_broadcast(ts)

    # ---------------------------------------------------------------- forward
    def forward(self, *inputs, **kwargs):
        if self.reducer is not None and torch.is_grad_enabled() and self.module.training:
            if self._iteration == 1 and not self._rebuilt:
                if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                    # a re-plan inside a hipGraph capture would allocate and zero the new bucket
                    # buffers as graph nodes (a fill re-run on every replay), and graphs captured
                    # later would hold other buffers than this one: keep the first plan (warm up
                    # with two eager steps to get the ready-order one, as engine / bench do)
                    self._rebuilt = True
                else:
                    self._rebuild_buckets()
            self.reducer.prepare_for_backward(self._sync_enabled)
            self._iteration += 1
        if self._buffers_need_sync and self.comm.active and self.require_forward_param_sync:
            bufs = [b for b in self.module.buffers()]
            if bufs:
                self._flat_broadcast(bufs)
        out = self.module(*inputs, **kwargs)
        # torch's _post_forward (distributed.py:1604-1617): the next forward broadcasts the
        # buffers only after a forward whose backward will sync (grad enabled, not no_sync)
        self.require_forward_param_sync = torch.is_grad_enabled() and self._sync_enabled
        return out

    def _rebuild_buckets(self):
        """Re-plan buckets in the order grads became ready during iteration 1."""
        self._rebuilt = True
        order = list(self.reducer.ready_order())
        if len(order) != len(self._params) or self.find_unused_parameters:
            return
        buckets = compute_bucket_assignment(self._params, self.bucket_cap_bytes, self.first_bucket_bytes, order)
        if buckets != [list(b) for b in self.reducer.bucket_indices()]:
            self.reducer.set_buckets(buckets)

    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = old

    # ------------------------------------------------ deferred grad averaging
    def defer_grad_sync_to(self, optimizer) -> bool:
        """Opt-in: let ``optimizer`` average the gradients instead of the reducer.

        At the end of backward the buckets are left holding this rank's
        gradients.  The fused AMP-SGD step (optim/sgd.py, GradScaler fast path)
        then exchanges them with the peers inside its own kernel over the xGMI
        engine (csrc/kernels/optim.hip, XG variant): no all-reduce launch.  Any
        other gradient consumer of ``optimizer`` (``step()``, ``GradScaler.unscale_``)
        first runs the bucket all-reduces (``reducer.flush_deferred``), so results
        never change, only the launch count.  ``.grad`` read directly between
        ``backward()`` and the optimizer step is therefore rank-local.

        Enabled only when the communicator has the xGMI engine, every optimizer
        parameter belongs to this module, and the gradients fit one exchange.
        ``DPA_FUSED_GRAD=0`` disables it.  Returns whether it was enabled.
        """
        if os.environ.get("DPA_FUSED_GRAD", "1") == "0" or self.reducer is None or not self.gradient_as_bucket_view:
            return False  # (the fused consumer writes the averaged gradients into the bucket views)
        xc = getattr(self.comm, "xgmi", None)
        if xc is None or not hasattr(optimizer, "fused_amp_step"):
            return False
        if (os.environ.get("DPA_SHARED_GPU") == "1" and self.comm.world_size > 2
                and os.environ.get("DPA_FUSED_GRAD") != "1"):
            # 3+ ranks sharing one GPU: every rank's AMP workgroups spin on the peers' rows,
            # and the ranks' launches need not be resident together on the one card (the
            # SyncBN sites are gated the same way: ops/convnet_fused._fused_site_engine).
            # Round 4's one stalled W=4 rehearsal (profiles/r4zz_*) had all four ranks inside
            # device work; with one rank per GPU this never applies.  DPA_FUSED_GRAD=1 forces it.
            return False
        opt_params = [p for g in optimizer.param_groups for p in g["params"]]
        if {id(p) for p in opt_params} != {id(p) for p in self._params}:
            return False
        n = sum((p.numel() + 3) // 4 * 4 for p in self._params)  # float4 granules, as the kernel counts
        if n > min(int(xc.max_bytes) // 4, int(_load_ext().optim.amp_sgd_xg_max())):
            return False
        self.reducer.set_defer(True)
        optimizer._deferred_ddp = (self.reducer, xc)
        return True

    def set_slab_sink(self, optimizer) -> bool:
        """Let ``optimizer`` also sum the wrapped model's deferred weight-gradient slab
        (models/convnet.py ``set_slab_sink``) under DDP.  Valid only while this reducer
        defers the average to that optimizer (``defer_grad_sync_to``) with zero-copy
        buckets: its hooks then read no gradient values, and the fused launch sums the slab
        and exchanges the result with the other gradients.  The reducer is told to fail
        loudly should a bucket ever need packing.  Returns whether it was enabled."""
        d = getattr(optimizer, "_deferred_ddp", None)
        # find_unused_parameters: a bucket holding an unused parameter is never tiled by the
        # fused gradient buffer, so the slab's required in-place bucket could not exist
        if (d is None or d[0] is not self.reducer or self.find_unused_parameters
                or not hasattr(self.module, "set_slab_sink")
                or os.environ.get("DPA_REDUCER_ZERO_COPY", "1") == "0"):
            return False
        if not self.module.set_slab_sink(optimizer):
            return False
        self.reducer.set_require_inplace(True)
        return True

    # -------------------------------------------------------------- utilities
    def bucket_sizes_bytes(self) -> list[int]:
        if self.reducer is None:
            return []
        return [t.numel() * t.element_size() for t in self.reducer.bucket_tensors()]
