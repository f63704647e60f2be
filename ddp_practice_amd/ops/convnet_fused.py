"""The whole ConvNet forward/backward as ONE autograd op (csrc/kernels/convnet_fused.hip).

Fusing across the layer boundaries of /root/reference/origin_main.py:9-31
removes launches that exist only because torch runs one module at a time:

  forward  (train): conv1(+BN1 sums, packs conv2's bf16 weight tiles) | BN1-ReLU-pool1 -> conv2 (+BN2 sums)
                    | BN2-ReLU-pool2 -> fc
                    = 3 launches for the model (per-layer ops: 6, torch: ~14 + host syncs)
  backward:         fc bwd (+BN2 sums) | BN2 bwd -> conv2 dgrad (+BN1 sums) | BN2 bwd -> conv2 wgrad
                    | BN1 bwd -> conv1 wgrad | weight-grad sums = 5 launches
                    (per-layer ops: 10, torch: ~20)

Every BatchNorm backward is applied while staging the operand of the next
GEMM (the conv-output gradient never exists in HBM), and its reductions are
emitted by the kernel that produced the pooled gradient.  With SyncBN
(``comm`` active) over the xGMI engine, each consuming kernel exchanges the
per-channel sums with its peers itself (csrc/comm/xsite.h): no collective
launch between the kernels.  Over any other communicator the partial sums are
all-reduced between the kernels (one small collective each: 2 forward,
2 backward).  Parameter gradients are views of one output buffer.
"""
from __future__ import annotations

import os

import torch

from .._ext import load as _load_ext


def _mods():
    C = _load_ext()
    return C.convblock, C.convnet


def supported(model, x: torch.Tensor) -> bool:
    if not x.is_cuda or x.dim() != 4 or tuple(x.shape[1:]) != (1, 28, 28):
        return False
    l1, l2, fc = model.layer1, model.layer2, model.fc
    for seq, cin, cout in ((l1, 1, 16), (l2, 16, 32)):
        conv, bn = seq[0], seq[1]
        if (conv.in_channels, conv.out_channels, conv.kernel_size, conv.stride, conv.padding) != \
                (cin, cout, (5, 5), (1, 1), (2, 2)) or conv.bias is None or conv.groups != 1:
            return False
        if not (bn.track_running_stats and bn.affine):
            return False
        if not isinstance(seq[2], torch.nn.ReLU) or not isinstance(seq[3], torch.nn.MaxPool2d):
            return False
    n, b = fc.out_features, x.shape[0]
    # head backward keeps dlogits, one channel of fc.weight and of the pooled features in LDS (64 KB)
    return fc.in_features == 32 * 49 and fc.bias is not None and 1 <= n <= 64 and b * (n + 49) + n * 49 <= 16384


_RESIDENT: dict = {}
_SPLIT_BWD2 = os.environ.get("DPA_SPLIT_BWD2", "0") == "1"
_SPLIT_WGRAD1 = os.environ.get("DPA_SPLIT_WGRAD1", "1") == "1"  # merged launch measured slower (15.0 vs 10.9 us)
# conv1 wgrad + conv2 slab sums in one launch even without a slab sink (A/B; then a conv1-only sum launch)
_WGRAD1_SLAB2 = os.environ.get("DPA_WGRAD1_SLAB2", "0") == "1"
# conv1's weight gradient deferred into the optimizer's fused launch (5 launches per step):
# measured no faster than the two launches it merges (54.2-54.6 vs 54.1-54.2 us/step,
# profiles/r4h_defer_wgrad1_ab.txt): the in-launch producer -> slab-owner hand-off (write-
# through rows, arrival counter, polling) costs ~3 us, more than the kernel boundary it
# removes; round 6, with the pre-checked step it gives up: 0.0516 vs 0.0482 ms
# (profiles/r6az_defer_wgrad1_ab.txt).  Opt-in: DPA_DEFER_WGRAD1=1
_DEFER_WGRAD1 = os.environ.get("DPA_DEFER_WGRAD1", "0") == "1"
# producer-side gradient checks instead of the fused AMP step's grid barrier (single rank);
# DPA_PRECHECK=0: the barrier (A/B runs)
_PRECHECK = os.environ.get("DPA_PRECHECK", "1") != "0"
_CAS_OK: dict = {}


def _wgrad1_deferrable(B: int, dtype: torch.dtype, opt) -> bool:
    """convnet.convnet_amp_step can run this batch size / dtype on this device (its AMP
    workgroups co-resident) and the optimizer's step takes the small fused path.

    Not for ranks sharing one GPU (DPA_SHARED_GPU=1, bench.py --share-gpu): the launch's
    ~470 workgroups per rank wait on the peers' exchange inside the kernel, and two ranks'
    launches do not fit the card together (a peer's workgroups could never be placed)."""
    if os.environ.get("DPA_SHARED_GPU") == "1" and getattr(opt, "_deferred_ddp", None) is not None:
        return False
    if not getattr(opt, "small_fusable", lambda: False)():
        return False
    gran = sum((p.numel() + 3) // 4 for g in opt.param_groups for p in g["params"])
    key = (B, dtype, gran)
    if key not in _CAS_OK:
        _CAS_OK[key] = bool(_load_ext().convnet.convnet_amp_step_ok(B, gran, dtype))
    return _CAS_OK[key]


def _fused_site_engine(comm, batch: int, dtype: torch.dtype):
    """The communicator's xGMI engine when SyncBN may exchange its sums inside the
    kernels (csrc/comm/xsite.h), else None (all-reduces between the launches).

    Every workgroup of such a launch polls the peers' rows, so the launch is only
    taken when all its workgroups fit on the device at once (occupancy x CUs,
    ``convnet.sites_resident``); DPA_FUSED_SYNC=0 forces the launch-per-collective
    path (A/B runs).

    The residency check is per rank, which is what matters with one rank per GPU.  Ranks
    SHARING one GPU (DPA_SHARED_GPU=1, bench.py --share-gpu) need all their launches'
    workgroups resident together: at batch 32 that holds for 2 ranks but not for 3 or 4,
    which then stall in the exchange (with batch 8 they complete;
    profiles/r2d_fused_sync_multirank.txt).  So 3+ ranks sharing a GPU take the
    launch-per-collective path unless DPA_FUSED_SYNC=1 forces the sites."""
    flag = os.environ.get("DPA_FUSED_SYNC")
    if flag == "0":
        return None
    if flag != "1" and os.environ.get("DPA_SHARED_GPU") == "1" and getattr(comm, "world_size", 1) > 2:
        return None
    xc = getattr(comm, "xgmi", None)
    if xc is None:
        return None
    key = (batch, dtype)
    if key not in _RESIDENT:
        _RESIDENT[key] = bool(_load_ext().convnet.sites_resident(batch, dtype))
    return xc if _RESIDENT[key] else None


class PreCE:
    """The loss a head-step launch already computed for (logits, labels, scale): the
    ``cross_entropy`` call finds it here and launches nothing (ops/head.py)."""

    __slots__ = ("target", "ignore_index", "smoothing", "scale", "loss", "dlog", "dls")

    def __init__(self, target, ignore_index, smoothing, scale, loss, dlog, dls):
        self.target, self.ignore_index, self.smoothing = target, ignore_index, smoothing
        self.scale, self.loss, self.dlog, self.dls = scale, loss, dlog, dls


_HEAD_OK: dict = {}
_HEAD_SPEC = os.environ.get("DPA_HEAD_SPEC", "1") != "0"  # 0: no speculative head backward (A/B)


def _head_step_ok(B: int, N: int, dtype: torch.dtype) -> bool:
    """The one-launch head (csrc/kernels/convnet_head.hip) handles this shape and its 32
    workgroups are co-resident.  DPA_HEAD_STEP=0 forces the three-launch head (A/B)."""
    if os.environ.get("DPA_HEAD_STEP", "1") == "0":
        return False
    H = _load_ext().convnet_head
    if not H.supported(B, N):
        return False
    if dtype not in _HEAD_OK:
        _HEAD_OK[dtype] = bool(H.resident(dtype))
    return _HEAD_OK[dtype]


class ConvNetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, g1, be1, w2, b2, g2, be2, wfc, bfc, bufs, training, moms, epss, comm, cdtype,
                labels=None, ce_cfg=(-100, 0.0), holder=None, state=None, gather=None, wcnt=None, sink=None):
        cb, cn = _mods()
        rm1, rv1, nbt1, rm2, rv2, nbt2 = bufs
        m1, m2 = (-1.0 if m is None else float(m) for m in moms)
        e1, e2 = (float(e) for e in epss)
        x = x.to(cdtype).contiguous()
        B = x.shape[0]
        dev = x.device
        N = wfc.shape[0]
        sync = comm is not None and comm.active and training
        # SyncBN sums exchanged inside the consuming kernels when the xGMI engine is up
        xc = _fused_site_engine(comm, B, cdtype) if sync else None
        y1 = torch.empty((B, 16, 28, 28), dtype=cdtype, device=dev)
        y2 = torch.empty((B, 32, 14, 14), dtype=cdtype, device=dev)
        logits = torch.empty((B, N), dtype=cdtype, device=dev)
        # layer-2 weights pre-packed (low precision, LDS tile layouts) by the conv1 launch
        wpk_f = torch.empty(cn.W2F_LEN, dtype=cdtype, device=dev)
        wpk_d = torch.empty(cn.W2D_LEN, dtype=cdtype, device=dev)
        fstats1 = torch.empty(cb.stats_len(16), dtype=torch.float32, device=dev)
        fstats2 = torch.empty(cb.stats_len(32), dtype=torch.float32, device=dev)
        if training:
            fslab1 = torch.empty(cb.fwd_rows(1, 16, 28, 28, B) * cb.fslab_row(16), dtype=torch.float32, device=dev)
            # conv2's workgroups per image depend on the dtype (convnet_fused.hip fwd2_split)
            fslab2 = torch.empty(B * cn.fwd2_split(cdtype == torch.float32) * cb.fslab_row(32), dtype=torch.float32,
                                 device=dev)
            # pooled maps, argmax|relu index and xhat at the argmax of both blocks (for the backward)
            p1 = torch.empty((B, 16, 14, 14), dtype=cdtype, device=dev)
            idx1 = torch.empty((B, 16, 14, 14), dtype=torch.uint8, device=dev)
            xh1 = torch.empty((B, 16, 14, 14), dtype=cdtype, device=dev)
            p2 = torch.empty((B, 32 * 49), dtype=cdtype, device=dev)
            idx2 = torch.empty((B, 32 * 49), dtype=torch.uint8, device=dev)
            xh2 = torch.empty((B, 32 * 49), dtype=cdtype, device=dev)
            if gather is not None:  # the batch gather runs inside conv1 (data/loader.py defer=True)
                imgs, lbls, order, ctr, lab_out, gsc, gsh = gather
                cn.conv1_fwd_pack_gather(x, w1, b1, y1, fslab1, fstats1, rm1, w2, wpk_f, wpk_d, imgs, lbls, order,
                                         ctr, lab_out, gsc, gsh)
            else:
                cn.conv1_fwd_pack(x, w1, b1, y1, fslab1, fstats1, rm1, w2, wpk_f, wpk_d)
            if sync and xc is None:
                comm.all_reduce_(fslab1)
            cn.conv2_fwd(y1, fslab1, fstats1, g1, be1, rm1, rv1, nbt1, m1, e1, True, w2, b2, y2, fslab2, fstats2,
                         rm2, p1, idx1, xh1, wpk_f, xc)
            if sync and xc is None:
                comm.all_reduce_(fslab2)
            ctx.spec = None
            ctx.chk = ctx.chk_scale = None
            if labels is not None and state is not None and _head_step_ok(B, N, cdtype):
                # labels known now (paired by the device loader): head forward + loss (+ the head
                # backward when a GradScaler will seed it with its scale) in one launch
                from .head import seed_scale

                scale = seed_scale(dev) if _HEAD_SPEC else None
                f32 = dict(dtype=torch.float32, device=dev)
                loss_buf = torch.empty(2, **f32)
                dlog = torch.empty((B, N), **f32)
                dls = torch.empty((B, N), dtype=cdtype, device=dev) if scale is not None else None
                spec = None
                if scale is not None:
                    # the row backward runs in this launch: dp2 and one row of BN2 backward
                    # sums per image; the fc weight gradient follows in the conv2 backward
                    dp2 = torch.empty_like(p2)
                    bsum2 = torch.empty(B * 64, **f32)
                    spec = (dls, dp2, bsum2)
                    # pre-checked gradients (slab sink; one rank, or the DDP average inside the
                    # AMP step over the xGMI engine): this launch clears the check word the
                    # backward's producers set (optim/sgd.py set_prechecked)
                    # Only for a GradScaler's scale (fp32's unit seed has no step to pre-check),
                    # and only where the producers' row bound FLT_MAX / W uses the world of the
                    # gradient exchange: the SyncBN site engine's (xc), or one rank.  Plain BN
                    # under a deferring DDP (--no-sync-bn: no xc, DDP world > 1) keeps the barrier.
                    from .head import _UNIT

                    ddp = getattr(sink, "_deferred_ddp", None) if sink is not None else None
                    ddp_world = int(ddp[1].world_size) if ddp is not None and ddp[1] is not None else 1
                    chk = None
                    if (sink is not None and _PRECHECK and scale is not _UNIT.get(dev)
                            and (xc is not None or (not sync and ddp_world == 1))
                            and hasattr(sink, "set_prechecked")):
                        sink.clear_prechecked()  # the device word is reset below
                        chk = sink.grad_chk(2, dev)
                    ctx.chk, ctx.chk_scale = chk, (scale if chk is not None else None)
                    _load_ext().convnet_head.head_step(
                        y2, fslab2, fstats2, g2, be2, rm2, rv2, nbt2, m2, e2, wfc, bfc, logits, p2, idx2, xh2, labels,
                        int(ce_cfg[0]), float(ce_cfg[1]), scale, state, loss_buf, dlog, dls, dp2, bsum2, xc, chk)
                else:
                    _load_ext().convnet_head.head_step(
                        y2, fslab2, fstats2, g2, be2, rm2, rv2, nbt2, m2, e2, wfc, bfc, logits, p2, idx2, xh2, labels,
                        int(ce_cfg[0]), float(ce_cfg[1]), None, state, loss_buf, dlog, None, None, None, xc, None)
                ctx.spec = spec
                if holder is not None:
                    holder["ce"] = PreCE(labels, int(ce_cfg[0]), float(ce_cfg[1]), scale, loss_buf, dlog, dls)
            else:
                cn.head_fwd(y2, fslab2, fstats2, g2, be2, rm2, rv2, nbt2, m2, e2, True, wfc, bfc, logits, p2, idx2,
                            xh2, xc)
            ctx.save_for_backward(x, wpk_d, wfc, g1, g2, y1, p1, idx1, xh1, fstats1, y2, p2, idx2, xh2, fstats2)
        else:
            cn.conv1_fwd_pack(x, w1, b1, y1, None, None, None, w2, wpk_f, wpk_d)
            cn.conv2_fwd(y1, None, fstats1, g1, be1, rm1, rv1, nbt1, m1, e1, False, w2, b2, y2, None, fstats2, rm2,
                         None, None, None, wpk_f, None)
            cn.head_fwd(y2, None, fstats2, g2, be2, rm2, rv2, nbt2, m2, e2, False, wfc, bfc, logits, None, None,
                        None, None)
        ctx.training = training
        ctx.wcnt = wcnt
        ctx.sink = sink
        ctx.w1b1 = (w1, b1) if sink is not None else None
        ctx.l12 = (w1, b1, g1, be1, w2, b2) if sink is not None else None
        ctx.allp = (w1, b1, g1, be1, w2, b2, g2, be2, wfc, bfc) if sink is not None else None
        ctx.sync = sync
        ctx.comm = comm
        ctx.xc = xc
        ctx.eps = (e1, e2)
        ctx.shapes = (w1.shape, w2.shape, wfc.shape)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        if not ctx.training:
            raise RuntimeError("ConvNetFn: backward through an eval-mode forward is not supported")
        cb, cn = _mods()
        x, wpk_d, wfc, g1, g2, y1, p1, idx1, xh1, fstats1, y2, p2, idx2, xh2, fstats2 = ctx.saved_tensors
        e1, e2 = ctx.eps
        comm, sync, xc = ctx.comm, ctx.sync, ctx.xc
        dl = dlogits.to(y2.dtype).contiguous()
        B = y2.shape[0]
        dev = y2.device
        s_w1, s_w2, s_wfc = ctx.shapes
        n_w1, n_w2, n_wfc = s_w1.numel(), s_w2.numel(), s_wfc.numel()
        N = s_wfc[0]
        f32 = dict(dtype=torch.float32, device=dev)
        ctx_spec = ctx.spec
        # one output buffer for every parameter gradient (views handed to autograd);
        # [dW1 | db1] and [dW2 | db2] are the rows of the two weight-grad slabs
        # [dW1 | db1 | dbeta1 | dgamma1] = conv1's slab columns, then BN1's [S1 | S2] sums
        sizes = [n_w1, 16, 16, 16, n_w2, 32, 32, 32, n_wfc, N]
        out = torch.empty(sum(sizes), **f32)
        dw1, db1, dbe1, dg1, dw2, db2, dg2, dbe2, dwfc, dbfc = out.split(sizes)
        fc = (None, None, None, None)
        if ctx_spec is not None and dlogits.data_ptr() == ctx_spec[0].data_ptr() and \
                dlogits.dtype == ctx_spec[0].dtype:
            # the gradient is the one the head-step launch predicted (the GradScaler seeded
            # the loss with its scale): dp2 and the per-image BN2 sums are already computed;
            # the fc weight gradient runs in the conv2 backward launch below (extra workgroups)
            ctx.spec = None
            dls, dp2, bsum2 = ctx_spec
            del ctx_spec
            fc = (dls, p2, dwfc, dbfc)
            dgb = (dg2, dbe2)  # BN2 dgamma / dbeta from the summed rows, in the conv2 backward
        else:
            # 1. fc backward -> dp2, fc grads, BN2 sums (complete per channel on this rank)
            bsum2 = torch.empty(64, **f32)
            dp2 = torch.empty_like(p2)
            cn.head_bwd(dl, wfc, p2, idx2, xh2, dwfc, dbfc, dg2, dbe2, bsum2, dp2)
            dgb = (None, None)
        if sync and xc is None:
            gsum2, lsum2 = comm.all_reduce(bsum2), (bsum2 if dgb[0] is not None else None)
        else:
            gsum2, lsum2 = bsum2, None
        # Pre-checked gradients (single rank, slab sink, AMP): the producer launches below record
        # per workgroup whether a gradient they finish is non-finite once unscaled, so the fused
        # AMP step agrees on found_inf without its grid barrier (optim/sgd.py set_prechecked)
        sink0 = ctx.sink
        chk, cscale = getattr(ctx, "chk", None), getattr(ctx, "chk_scale", None)
        ctx.chk = ctx.chk_scale = None
        if sink0 is not None and hasattr(sink0, "set_prechecked"):
            sink0.clear_prechecked()  # an earlier backward's check no longer describes .grad
        if not (chk is not None and fc[0] is not None and not _SPLIT_BWD2 and not _DEFER_WGRAD1
                and all(p.grad is None for p in ctx.allp)):
            chk = cscale = None
        # 2+3. BN2 bwd -> {conv2 dgrad -> dp1 (+ BN1 partial sums), conv2 wgrad partials}: one launch
        #      (DPA_SPLIT_BWD2=1: the two as separate launches, A/B runs)
        dp1 = torch.empty((B, 16, 14, 14), dtype=y1.dtype, device=dev)
        bslab1 = torch.empty(cn.dgrad2_rows(B, y1.dtype == torch.float32) * 32, **f32)
        wslab2 = torch.empty(cn.wgrad_bn_rows(2, B) * (n_w2 + 32), **f32)
        if _SPLIT_BWD2:
            if dgb[0] is not None:  # the BN2 parameter grads from the rows (this rank's)
                rows = (lsum2 if lsum2 is not None else gsum2).view(-1, 64).sum(0)
                dbe2.copy_(rows[:32])
                dg2.copy_(rows[32:])
            cn.conv2_dgrad(wpk_d, y2, dp2, idx2, fstats2, gsum2, g2, e2, dp1, idx1, xh1, bslab1, xc)
            cn.conv_wgrad_bn(p1, y2, dp2, idx2, fstats2, gsum2, None, g2, e2, None, None, wslab2, xc)
            if fc[0] is not None:
                cn.fc_wgrad(*fc)
        else:
            cn.conv2_bwd(wpk_d, y2, dp2, idx2, fstats2, gsum2, g2, e2, dp1, idx1, xh1, bslab1, p1, wslab2, xc,
                         lsum2, dgb[0], dgb[1], *fc, chk)
        # 4+5. BN1 bwd -> conv1 wgrad partials (+ dgamma1 / dbeta1 from the local sums), and the
        #      column sums of both weight-grad slabs -> [dW1 | db1], [dW2 | db2]: one launch
        #      (DPA_SPLIT_WGRAD1=1: wgrad launch + a separate reduction launch, A/B runs)
        wslab1 = torch.empty(cn.wgrad_bn_rows(1, B) * (n_w1 + 16), **f32)
        if sync and xc is None:
            gsum1, lsum1, xc1 = comm.all_reduce(bslab1), bslab1, None
        else:
            gsum1, lsum1, xc1 = bslab1, None, xc
        out1, out2 = out.narrow(0, 0, n_w1 + 16), out.narrow(0, n_w1 + 48, n_w2 + 32)
        out0 = out.narrow(0, n_w1 + 16, 32)  # [dbeta1 | dgamma1]
        sink = ctx.sink
        w1b1, l12 = ctx.w1b1, ctx.l12
        ctx.w1b1 = ctx.l12 = None
        if sink is not None:
            sink.flush_slab()  # an earlier backward's sums first (they may be accumulated into)
            # a gradient region is left to the optimizer's fused step only when autograd will
            # hand its views to .grad as they are (no accumulation into an existing .grad)
            if any(p.grad is not None for p in w1b1):
                sink = None
        if (sink is not None and _DEFER_WGRAD1 and hasattr(sink, "defer_wgrad1")
                and all(p.grad is None for p in l12) and _wgrad1_deferrable(B, x.dtype, sink)):
            # the conv1 weight gradient itself, BN1's and conv2's column sums: all computed
            # inside the optimizer's fused launch (convnet.convnet_amp_step); the backward
            # launches nothing more.  Any other gradient reader flushes first (optim.SGD)
            # (only regions of `out` other than the returned views: a second reference to a
            # returned gradient makes autograd copy it into .grad now, before it is computed)
            sink.defer_wgrad1(dict(x=x, y1=y1, dp1=dp1, idx1=idx1, fstats1=fstats1, gsum1=gsum1, lsum1=lsum1, g1=g1,
                                   e1=e1, wslab1=wslab1, out1=out1, bn1=lsum1 if lsum1 is not None else gsum1,
                                   out0=out0, wslab2=wslab2, out2=out2, xc1=xc1))
        elif sink is not None or _WGRAD1_SLAB2:
            # conv1 wgrad partials + the conv2 slab's column sums in one launch; the conv1
            # slab's sums run inside the fused AMP-SGD launch (optim.SGD.defer_slab) or next
            if sink is None:
                chk = cscale = None
            cn.conv1_wgrad_slab2(x, y1, dp1, idx1, fstats1, gsum1, lsum1, g1, e1, dg1, dbe1, wslab1, wslab2, out2,
                                 xc1, chk)
            if sink is not None:
                sink.defer_slab(wslab1, out1)
                if chk is not None:
                    sink.set_prechecked(chk, cscale, out)
            else:
                cb.slab_reduce(wslab1, n_w1 + 16, out1)
        elif _SPLIT_WGRAD1 or ctx.wcnt is None:
            cn.conv_wgrad_bn(x, y1, dp1, idx1, fstats1, gsum1, lsum1, g1, e1, dg1, dbe1, wslab1, xc1)
            cb.slab_reduce(wslab1, n_w1 + 16, out1, wslab2, n_w2 + 32, out2)
        else:
            cnt = ctx.wcnt
            gslab1 = torch.empty((cn.wgrad1_counters(B) - 1) * (n_w1 + 16), **f32)
            cn.wgrad1_reduce(x, y1, dp1, idx1, fstats1, gsum1, lsum1, g1, e1, dg1, dbe1, wslab1, gslab1, out1,
                             wslab2, out2, cnt, xc1)
        return (None, dw1.view(s_w1), db1, dg1, dbe1, dw2.view(s_w2), db2, dg2, dbe2, dwfc.view(s_wfc), dbfc,
                None, None, None, None, None, None, None, None, None, None, None, None, None)


def convnet_forward(model, x, comm=None, cdtype=None):
    """Run the reference ConvNet module tree through the fused op.

    When ``x`` carries the labels of its batch (``DeviceLoader.fill_`` pairs them) and
    the model trains, the head, the loss and the head backward run as one launch; the
    returned logits then carry the computed loss for ``cross_entropy`` (ops/head.py).
    """
    if cdtype is None:
        from ..amp import compute_dtype

        cdtype = compute_dtype(x)
    l1, l2, fc = model.layer1, model.layer2, model.fc
    c1, bn1, c2, bn2 = l1[0], l1[1], l2[0], l2[1]
    training = bn1.training
    if bn1.training != bn2.training:
        raise RuntimeError("fused ConvNet: both BatchNorms must be in the same mode")
    bufs = (bn1.running_mean, bn1.running_var, bn1.num_batches_tracked,
            bn2.running_mean, bn2.running_var, bn2.num_batches_tracked)
    gather = getattr(x, "_dpa_gather", None)
    if gather is not None:
        if training and x.dtype == cdtype and x.is_contiguous():
            x._dpa_gather = None  # consumed by conv1 below
        else:
            from ..data.loader import flush_pending

            flush_pending(x)
            gather = None
    labels = getattr(x, "_dpa_labels", None) if training else None
    holder, state = None, None
    if labels is not None:
        if labels.shape != (x.shape[0],) or labels.dtype != torch.int64 or labels.device != x.device:
            labels = None
        else:
            holder = {}
            state = getattr(model, "_dpa_head_state", None)
            if state is None or state.device != x.device:
                # ticket / flag / error words of the head-step launch (zeroed once; the
                # kernel re-arms them itself, so graph replays need no reset)
                state = torch.zeros(4, dtype=torch.int64, device=x.device)
                model._dpa_head_state = state
    wcnt = None
    if training:
        # tickets of the in-launch weight-grad reduction (zeroed once, re-armed by the kernel)
        n = _load_ext().convnet.wgrad1_counters(x.shape[0])
        wcnt = getattr(model, "_dpa_wgrad_cnt", None)
        if wcnt is None or wcnt.numel() < n or wcnt.device != x.device:
            wcnt = torch.zeros(max(n, 64), dtype=torch.int32, device=x.device)
            model._dpa_wgrad_cnt = wcnt
    out = ConvNetFn.apply(x, c1.weight, c1.bias, bn1.weight, bn1.bias, c2.weight, c2.bias, bn2.weight, bn2.bias,
                          fc.weight, fc.bias, bufs, training, (bn1.momentum, bn2.momentum), (bn1.eps, bn2.eps),
                          comm, cdtype, labels, (-100, 0.0), holder, state, gather, wcnt,
                          getattr(model, "_dpa_slab_sink", None) if training else None)
    if holder:
        out._dpa_pre_ce = holder.get("ce")
    return out
