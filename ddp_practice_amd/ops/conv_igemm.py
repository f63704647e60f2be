"""Forward convolution on the hand-written NHWC implicit-GEMM MFMA kernel
(csrc/kernels/conv_igemm.hip) with the following BatchNorm's statistics fused
into its epilogue (ResNet-50 stress model, models/resnet.py).

``conv_forward(x, weight, stride, pad, cdtype, bn)`` returns the channels_last
output and, when ``bn`` is a training BatchNorm, the statistics vector that
``ops/bn_nhwc.bn_act(..., stats=...)`` consumes instead of running its own
statistics pass over the activation (sums around the running mean, row count,
shift copy; num_batches_tracked bumped in the same launch).
"""
from __future__ import annotations

import os

import torch

from .._ext import load as _load_ext
from .bn_nhwc import bn_comm, sync_site

_CL = torch.channels_last
ENABLED = os.environ.get("DPA_IGEMM", "1") != "0"  # 0: MIOpen / hipBLASLt forward + separate stats (A/B)


def _K():
    return _load_ext().conv_igemm


class _StatWS:
    """Per-device partial rows + tickets of the in-launch statistics tree (stream-ordered
    reuse: every launch re-arms the tickets it used)."""

    _by_dev: dict = {}

    @classmethod
    def get(cls, dev: torch.device, M: int, K: int):
        k = _K()
        need_p, need_t = int(k.stat_part_len(M, K)), int(k.stat_tickets_len(M, K))
        ws = cls._by_dev.get(dev)
        if ws is None or ws[0].numel() < need_p or ws[1].numel() < need_t:
            part = torch.empty(max(need_p, 1 << 20), dtype=torch.float32, device=dev)
            tickets = torch.zeros(max(need_t, 1 << 12), dtype=torch.int32, device=dev)
            ws = cls._by_dev[dev] = (part, tickets)
        return ws


def usable(x: torch.Tensor, weight: torch.Tensor, cdtype: torch.dtype) -> bool:
    return (ENABLED and x.is_cuda and cdtype in (torch.bfloat16, torch.float16) and weight.dim() == 4
            and bool(_K().supported(weight.shape[1], weight.shape[0])))


G1X1 = os.environ.get("DPA_G1X1", "1") != "0"  # 1x1 convs on conv_glds_kernel (0: general kernel, A/B)


def dgrad_1x1_here(K: int, OH: int) -> bool:
    """1x1 data gradients that run on the hand-written kernels: every one on the glds 1x1
    GEMM kernel (network total 1150 us vs hipBLASLt 1485 us at bs 128,
    profiles/r3_g1x1_bench.txt); with DPA_G1X1=0 only the shapes where the general
    implicit-GEMM kernel beats hipBLASLt (<= 512 gradient channels at 14x14 and above)."""
    return ENABLED and (G1X1 or (K <= 512 and OH >= 14))


def conv_acc(x: torch.Tensor, w: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """y += conv1x1(x, w) in place (stride 1): the data gradient accumulated onto a
    residual gradient already in y (ops/conv1x1.py GradTap)."""
    _K().conv_fwd(x, w, y, 1, 0, accumulate=True)
    return y


def conv_fwd(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int, bn=None, aux=None, mode: int = 0):
    """y = conv(x, w) on the implicit-GEMM kernel; x, w channels_last in the compute dtype.
    With ``bn`` (a training BatchNorm module): also its statistics, returned as the second
    value (None otherwise).  ``aux`` ([N, K, OH/2, OW/2] channels_last): added into the
    even output pixels (a stride-2 1x1 conv's data gradient folded in).  ``mode``:
    MODE_STEM (x, w from :func:`stem_conv`'s pack, R = 7 semantics)."""
    N, C, H, W = x.shape
    K, _, R, S = w.shape
    if mode == _K().MODE_STEM:
        R = S = 7
    OH, OW = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
    y = torch.empty((N, K, OH, OW), dtype=x.dtype, device=x.device, memory_format=_CL)
    if bn is None:
        _K().conv_fwd(x, w, y, stride, pad, mode=mode, aux=aux)
        return y, None
    part, tickets = _StatWS.get(x.device, N * OH * OW, K)
    stats = torch.empty(3 * K + 4, dtype=torch.float32, device=x.device)
    # SyncBN: the statistics finishers exchange with the peers (the BN then skips its all-reduce)
    xc = sync_site(bn_comm(bn))
    _K().conv_fwd(x, w, y, stride, pad, part, tickets, stats, bn.running_mean, bn.num_batches_tracked, mode=mode,
                  aux=aux, xc=xc)
    return y, stats


def dgrad_bn(dy: torch.Tensor, wt: torch.Tensor, bt, acc: torch.Tensor | None = None,
             pad: int = 0) -> torch.Tensor | None:
    """Stride-1 data gradient dx = conv(dy, wt, pad) (+= acc, the tapped residual gradient;
    1x1 only) whose epilogue also takes the backward sums of the BatchNorm that produced the
    conv's input (``bt``: ops/bn_nhwc.BNTap, filled by that BN's forward).  ``wt``: the
    flipped transposed filter, ``pad`` = R - 1 - the forward padding.  Stores the sums in
    ``bt`` and returns dx; None when the shapes do not allow it (the BN then runs its own
    statistics pass)."""
    if bt is None or not G1X1:
        return None
    bx = bt.x  # the producing BN's saved input (None once its node is gone)
    if bx is None:
        return None
    if (acc is None) != (bt.act == 2):  # act 1 (ReLU after a residual add) <-> accumulated dx
        return None
    R, S = wt.shape[2], wt.shape[3]
    if (R, S) != (1, 1) and (acc is not None or 2 * pad != R - 1 or R != S):
        return None
    N, _, H, W = dy.shape
    C = wt.shape[0]
    shape = (N, C, H, W)
    if tuple(bx.shape) != shape or bx.dtype != dy.dtype or not bx.is_contiguous(memory_format=_CL):
        return None
    if acc is not None and (tuple(acc.shape) != shape or not acc.is_contiguous(memory_format=_CL)):
        return None
    f32 = dict(dtype=torch.float32, device=dy.device)
    part, tickets = _StatWS.get(dy.device, N * H * W, C)
    out, dgamma, dbeta = torch.empty(2 * C, **f32), torch.empty(C, **f32), torch.empty(C, **f32)
    dx = acc if acc is not None else torch.empty(shape, dtype=dy.dtype, device=dy.device, memory_format=_CL)
    _K().conv_fwd(dy, wt, dx, 1, pad, part, tickets, accumulate=acc is not None, bn_x=bx,
                  bn_y=bt.y if bt.act == 1 else None, bn_save=bt.save, bn_gamma=bt.weight, bn_beta=bt.bias,
                  bn_out=out, bn_dgamma=dgamma, bn_dbeta=dbeta, xc=bt.xc)
    bt.sums = (out, dgamma, dbeta)
    bt.grad_ptr = dx.data_ptr()
    bt.grad_ver = dx._version
    return dx


def dgrad_s2(dy: torch.Tensor, wt: torch.Tensor, in_hw) -> torch.Tensor | None:
    """Data gradient of a 3x3 / stride-2 / pad-1 conv on the implicit-GEMM kernel
    (MODE_S2T: four output-parity sub-convolutions, csrc/kernels/conv_igemm.hip).
    ``wt``: the flipped transposed filter [Cin, Cout, 3, 3] channels_last; ``in_hw``: the
    forward input's (H, W).  None when the shape is not covered (odd input sizes)."""
    N, Kf, OH, OW = dy.shape
    H, W = in_hw
    if H != 2 * OH or W != 2 * OW:
        return None
    dx = torch.empty((N, wt.shape[0], H, W), dtype=dy.dtype, device=dy.device, memory_format=_CL)
    _K().conv_fwd(dy, wt, dx, 2, 1, mode=_K().MODE_S2T)
    return dx


def stem_usable(x: torch.Tensor, conv, cdtype: torch.dtype) -> bool:
    """The 7x7 / stride-2 / pad-3 stem over a 3-channel image runs on the kernel's
    MODE_STEM (the image needs no gradient: it is the network input)."""
    return (ENABLED and x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and not x.requires_grad
            and cdtype in (torch.bfloat16, torch.float16) and x.dtype in (torch.float32, cdtype)
            and conv.kernel_size == (7, 7) and conv.stride == (2, 2) and conv.padding == (3, 3)
            and conv.bias is None and conv.groups == 1 and conv.dilation == (1, 1)
            and conv.weight.dtype == torch.float32 and conv.weight.shape[0] % 64 == 0)


class StemConvFn(torch.autograd.Function):
    """ResNet stem on the implicit-GEMM kernel: one launch packs the image to 4-channel
    NHWC and the filter to the padded [K][8][8][4] space, one conv launch (+ the
    following BN's statistics); backward = the weight gradient only."""

    @staticmethod
    def forward(ctx, x, weight, cdtype, bn):
        N, _, H, W = x.shape
        K = weight.shape[0]
        x4 = torch.empty((N, 4, H, W), dtype=cdtype, device=x.device, memory_format=_CL)
        w4 = torch.empty((K, 4, 8, 8), dtype=cdtype, device=x.device, memory_format=_CL)
        _K().stem_pack(x.contiguous(), weight.contiguous(), x4, w4)
        y, stats = conv_fwd(x4, w4, 2, 3, bn, mode=_K().MODE_STEM)
        ctx.save_for_backward(x4)
        ctx.wshape = tuple(weight.shape)
        ctx.wparam = weight  # the leaf parameter (WgradBatch: is its .grad still unset?)
        ctx.set_materialize_grads(False)
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, *_):
        (x4,) = ctx.saved_tensors
        if dy is None:
            return None, None, None, None
        dy = dy.to(x4.dtype)
        dy = dy if dy.is_contiguous(memory_format=_CL) else dy.contiguous(memory_format=_CL)
        K = ctx.wshape[0]
        N, _, OH, OW = dy.shape
        sp = int(_K().wgrad_splits(N * OH * OW, K, 4, 8, 8))
        grad = torch.empty(ctx.wshape, dtype=torch.float32, device=dy.device)
        if WgradBatch.wants(ctx.wparam):
            slab = torch.empty(sp * K * 256, dtype=torch.float32, device=dy.device)
            WgradBatch.add(slab, grad, ctx.wparam,
                           _K().conv_wgrad(dy, x4, grad, 2, 3, slab, mode=_K().MODE_STEM, reduce=False))
        else:
            slab = _WgradWS.get(dy.device, sp * K * 256)
            _K().conv_wgrad(dy, x4, grad, 2, 3, slab, mode=_K().MODE_STEM)
        ctx.wparam = None
        return None, grad, None, None


def stem_conv(x: torch.Tensor, conv, cdtype: torch.dtype, bn=None):
    """(output channels_last in ``cdtype``, statistics of ``bn`` or None)."""
    return StemConvFn.apply(x, conv.weight, cdtype, bn if (bn is not None and bn.training) else None)


class WgradBatch:
    """Weight-gradient split-K reductions of a whole backward pass in ONE launch.

    Each implicit-GEMM weight gradient writes fp32 partial tiles (one per pixel split) that
    a reduction folds into the OIHW ``.grad``: 53 small launches per ResNet-50 step, ~9 us
    each, tail-bound (profiles/r5a_rn_steady.txt).  While ``active`` (set by the native
    ResNet-50 forward when no DDP reducer or peer rank can read the gradients mid-backward),
    a conv whose weight has no ``.grad`` yet (autograd then adopts the returned tensor
    without reading it) keeps its partials in a slab of its own and the reductions of the
    whole pass run in one launch from an end-of-backward callback (csrc/kernels/
    conv_igemm.hip wgrad_reduce_batch: the same association, bitwise the same gradients),
    before ``backward()`` returns.

    Opt-in (DPA_WGRAD_BATCH=1): measured slower on ResNet-50 (14.63 vs 14.52-14.56 ms/step,
    profiles/r5d_*): the reductions are bound by the ~1 GB of fp32 partials they re-read,
    not by launch count, and batched at the end of the backward those partials have left
    the 256 MB MALL that the per-conv reduction reads them from."""

    enabled = os.environ.get("DPA_WGRAD_BATCH", "0") == "1"
    active = False
    _pending: list = []

    @classmethod
    def wants(cls, wparam) -> bool:
        return cls.enabled and cls.active and wparam is not None and wparam.grad is None

    @classmethod
    def add(cls, slab: torch.Tensor, grad: torch.Tensor, wparam, geo) -> None:
        # no reference to ``grad`` is kept: autograd adopts a gradient tensor as ``.grad``
        # only while nothing else holds it (otherwise it clones it -- reading it now); the
        # flush finds it again as ``wparam.grad`` and checks it is the same memory
        cls._pending.append((slab, grad.data_ptr(), wparam, list(geo)))
        # one callback per deferral (the first flushes them all): a backward that raised
        # part-way leaves no stale "already queued" state behind
        torch.autograd.Variable._execution_engine.queue_callback(cls.flush)

    @classmethod
    def flush(cls) -> None:
        if not cls._pending:
            return
        p, cls._pending = cls._pending, []
        grads = [w.grad for _, _, w, _ in p]
        for (_, ptr, w, _), g in zip(p, grads):
            if g is None or g.data_ptr() != ptr:
                raise RuntimeError("WgradBatch: a deferred weight gradient was not adopted as .grad (a hook or "
                                   "accumulation read it before its reduction); set DPA_WGRAD_BATCH=0")
        _K().wgrad_reduce_batch([a for a, _, _, _ in p], grads, [c for _, _, _, c in p])


class _WgradWS:
    _by_dev: dict = {}

    @classmethod
    def get(cls, dev: torch.device, n: int):
        ws = cls._by_dev.get(dev)
        if ws is None or ws.numel() < n:
            ws = cls._by_dev[dev] = torch.empty(max(n, 1 << 22), dtype=torch.float32, device=dev)
        return ws


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, wshape, stride: int, pad: int, wparam=None) -> torch.Tensor:
    """fp32 OIHW weight gradient of a conv on the implicit-GEMM kernel (pixel-split
    partials reduced straight into the OIHW layout); dy, x channels_last.  ``wparam``: the
    weight parameter (the reduction may then join the pass's batch, :class:`WgradBatch`)."""
    K, C, R, S = wshape
    N, _, OH, OW = dy.shape
    sp = int(_K().wgrad_splits(N * OH * OW, K, C, R, S))
    grad = torch.empty(wshape, dtype=torch.float32, device=dy.device)
    if WgradBatch.wants(wparam):
        slab = torch.empty(sp * K * C * R * S, dtype=torch.float32, device=dy.device)
        WgradBatch.add(slab, grad, wparam, _K().conv_wgrad(dy, x, grad, stride, pad, slab, reduce=False))
        return grad
    slab = _WgradWS.get(dy.device, sp * K * C * R * S)
    _K().conv_wgrad(dy, x, grad, stride, pad, slab)
    return grad


class WeightPack:
    """One launch per forward that writes, for every implicit-GEMM conv of a network,
    the compute-dtype filter in the kernels' layout and, where the data gradient also
    runs on the kernel, its flipped transpose (csrc/kernels/conv_igemm.hip
    pack_weights_kernel) -- instead of 2-3 cast / flip / transpose copies per conv.

    ``convs``: (module, wants_dgrad_filter) pairs.  The buffers persist (the same
    addresses every step: graph-capturable); the tile table is rebuilt only when a
    weight tensor is replaced."""

    def __init__(self, convs, cdtype: torch.dtype):
        self.items = [(m, bool(d)) for m, d in convs]
        self.cdtype = cdtype
        self._key = None
        self._bufs: dict = {}
        self._table = None
        self._tiles = 0

    def _build(self, dev):
        rows, tiles = [], 0
        for m, want_d in self.items:
            w = m.weight
            K, C, R, S = w.shape
            wf = torch.empty((K, C, R, S), dtype=self.cdtype, device=dev, memory_format=_CL)
            wd = torch.empty((C, K, R, S), dtype=self.cdtype, device=dev, memory_format=_CL) if want_d else None
            self._bufs[id(m)] = (wf, wd)
            rows.append([w.data_ptr(), wf.data_ptr(), wd.data_ptr() if wd is not None else 0, K, C, R * S, tiles, 0])
            tiles += (K // 64) * (C // 64) * R * S
        self._table = torch.tensor(rows, dtype=torch.int64).reshape(-1).to(dev)
        self._tiles = tiles

    def run(self) -> dict:
        key = tuple(m.weight.data_ptr() for m, _ in self.items)
        if key != self._key:
            self._build(self.items[0][0].weight.device)
            self._key = key
        code = 0 if self.cdtype == torch.bfloat16 else 1
        _K().pack_weights(self._table, len(self.items), self._tiles, code)
        return self._bufs
