"""ResNet-50 (torchvision layout: same module tree, parameter names and
state_dict keys, 25,557,032 parameters) for the BASELINE.json stress config
"ResNet-50 on synthetic 3x224x224, world_size=8 AMP bf16 (stress MFMA conv +
all-reduce bucket fusion)".  The reference repository has no ResNet; the
architecture is He et al. 2015 with the v1.5 stride placement (stride on the
3x3 conv of each stage's first bottleneck), the variant torchvision ships.

Execution on a HIP device (``fused=True``): activations are bf16/f16/f32
``channels_last`` (NHWC in memory) end to end;
  * forward convolutions (1x1 and 3x3, any stride; C and Cout multiples of 64)
    run on the hand-written NHWC implicit-GEMM MFMA kernel, which also produces
    the following BatchNorm's batch statistics in its epilogue
    (csrc/kernels/conv_igemm.hip, ops/conv_igemm.py; DPA_IGEMM=0: library path);
  * the 7x7 / stride-2 stem (C = 3) runs on the same kernel's stem mode: the image
    is packed to 4-channel NHWC in one launch and the K space is (r, s, c) padded to
    8 x 8 x 4 (forward + statistics, and the weight gradient);
  * backward: every weight gradient and every 3x3 data gradient (stride 1, and
    stride 2 as four output-parity sub-convolutions) run on the implicit-GEMM
    kernel; 1x1 forwards and data gradients run on the glds-staged 1x1 GEMM kernel
    (conv_glds_kernel: 128-pixel tiles, operands global -> LDS by LDS-DMA).  A
    projection block's two input gradients (conv1 and downsample) are combined in
    the conv epilogue instead of by a separate add;
  * every BatchNorm runs on the native NHWC kernels with its ReLU and, for the
    last BN of a bottleneck, the residual add fused in (ops/bn_nhwc.py), as
    SyncBatchNorm when the module was converted (one small all-reduce each way);
  * max-pool 3x3/2 and the global average pool are native kernels; fc runs on the
    native MFMA linear kernels (ops/head.py).
On CPU the plain torch modules run (the same math; the CPU test tier).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..amp import autocast, compute_dtype
from ..ops import conv_igemm as _igemm
from ..ops.conv1x1 import GradTap, conv1x1
from ..ops.conv_nhwc import conv_nhwc


_PACKS: dict = {}  # id(module) -> this forward's packed filters (ops/conv_igemm.WeightPack)
_FUSE_BN_BWD = os.environ.get("DPA_FUSE_BN_BWD", "1") != "0"  # BNTap hand-off (0: own bwd_stats pass, A/B)
# bn1 -> the 3x3 conv2's data gradient: off by default -- the 3x3 epilogue's extra cost
# (+281 us over 13 launches) cancels the bwd_stats pass it removes (-297 us),
# profiles/r3s2h_resnet50_steady_bn1_fused.txt
_FUSE_BN1 = os.environ.get("DPA_FUSE_BN1", "0") == "1"
# a projection block's downsample BN applied inside bn3's residual add (ops/bn_nhwc.bn_res_bn)
_FUSE_DS_BN = os.environ.get("DPA_FUSE_DS_BN", "1") != "0"


def _conv(x: torch.Tensor, conv: nn.Conv2d, cdtype: torch.dtype, bn: nn.Module | None = None, tap=None,
          xtap=None, btap=None):
    """conv(x) -> (output, statistics of the following training BN ``bn`` when the conv
    kernel produced them, else None).  ``btap``: the BNTap of the BN that produced ``x``
    (a 1x1 conv's data gradient then also takes that BN's backward sums)."""
    want = bn if (bn is not None and bn.training) else None
    pk = _PACKS.get(id(conv))
    if conv.kernel_size == (1, 1) and conv.padding == (0, 0) and conv.groups == 1 and conv.bias is None:
        if want is None:
            return conv1x1(x, conv.weight, conv.stride[0], cdtype, tap, None, pk, xtap, btap), None
        return conv1x1(x, conv.weight, conv.stride[0], cdtype, tap, want, pk, xtap, btap)
    if conv.bias is None and conv.groups == 1 and conv.dilation == (1, 1):
        if want is None:
            return conv_nhwc(x, conv.weight, conv.stride, conv.padding, cdtype, None, pk, btap), None
        return conv_nhwc(x, conv.weight, conv.stride, conv.padding, cdtype, want, pk, btap)
    w = conv.weight.to(cdtype)
    out = F.conv2d(x, w, None if conv.bias is None else conv.bias.to(cdtype), conv.stride, conv.padding,
                   conv.dilation, conv.groups)
    return (out if out.is_contiguous(memory_format=torch.channels_last) else
            out.contiguous(memory_format=torch.channels_last)), None


def _multi_rank() -> bool:
    import torch.distributed as tdist

    from .. import distributed as ddist

    if tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1:
        return True
    try:
        return ddist.is_initialized() and ddist.get_world_size() > 1
    except Exception:  # noqa: BLE001 -- no facade state: a single process
        return False


def _comm_of(bn: nn.Module):
    from ..ops.bn_nhwc import bn_comm  # the same lookup the statistics-producing convs use

    return bn_comm(bn)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module | None = None):
        super().__init__()
        width = planes
        self.conv1 = nn.Conv2d(inplanes, width, kernel_size=1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, planes * self.expansion, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        return self.relu(out + identity)

    def forward_native(self, x: torch.Tensor, cdtype: torch.dtype, bt_in=None):
        """Native block forward; returns (y, the BNTap of bn3 or None).  ``bt_in``: the
        previous block's bn3 tap (the BN that produced ``x``)."""
        from ..ops.bn_nhwc import BNTap, bn_act

        train = self.bn3.training and torch.is_grad_enabled()
        grad_x = train and x.requires_grad and x.is_contiguous(memory_format=torch.channels_last)
        # identity blocks: conv1's dgrad GEMM accumulates the residual gradient (GradTap);
        # projection blocks: conv1 and the downsample conv share x's gradient (one of them
        # folds the other's product into its own, ops/conv1x1.Conv1x1Fn)
        tap = GradTap() if (grad_x and self.downsample is None) else None
        xtap = GradTap() if (grad_x and self.downsample is not None) else None
        # BN backward sums taken by the consuming conv's data-gradient epilogue
        # (ops/bn_nhwc.BNTap): bn2 -> conv3, and the previous block's bn3 -> this conv1
        # when this is an identity block (its dgrad then holds the whole gradient of x);
        # bn1 -> conv2 (stride 1) with DPA_FUSE_BN1=1
        bt_in = bt_in if tap is not None else None
        bt1 = BNTap() if train and _FUSE_BN1 and self.conv2.stride == (1, 1) else None
        bt2 = BNTap() if train and _FUSE_BN_BWD else None
        bt3 = BNTap() if train and _FUSE_BN_BWD else None
        # each conv hands the following BN its batch statistics (ops/conv_igemm.py)
        c1, st = _conv(x, self.conv1, cdtype, self.bn1, tap, xtap, bt_in)
        out = bn_act(c1, self.bn1, relu=True, comm=_comm_of(self.bn1), stats=st, btap=bt1)
        c2, st = _conv(out, self.conv2, cdtype, self.bn2, btap=bt1)
        out = bn_act(c2, self.bn2, relu=True, comm=_comm_of(self.bn2), stats=st, btap=bt2)
        identity = x
        cd = std = None
        if self.downsample is not None:
            conv, bn = self.downsample[0], self.downsample[1]
            cd, std = _conv(x, conv, cdtype, bn, None, xtap)
            if not _FUSE_DS_BN:
                identity = bn_act(cd, bn, relu=False, comm=_comm_of(bn), stats=std)
        c3, st = _conv(out, self.conv3, cdtype, self.bn3, btap=bt2)
        if cd is not None and _FUSE_DS_BN:
            # downsample BN applied inside the residual add (no normalised identity written)
            from ..ops.bn_nhwc import bn_res_bn

            y = bn_res_bn(c3, self.bn3, cd, self.downsample[1], comm=_comm_of(self.bn3), stats=st, rstats=std,
                          btap=bt3)
        else:
            y = bn_act(c3, self.bn3, res=identity, relu=True, comm=_comm_of(self.bn3), tap=tap, stats=st, btap=bt3)
        return y, bt3


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1000, amp_dtype: torch.dtype | None = None,
                 fused: bool = True):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0])
        self.layer2 = self._make_layer(128, layers[1], stride=2)
        self.layer3 = self._make_layer(256, layers[2], stride=2)
        self.layer4 = self._make_layer(512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)
        for m in self.modules():  # torchvision's initialisation
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        self.amp_dtype = amp_dtype
        self.fused = fused

    def _make_layer(self, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * Bottleneck.expansion, kernel_size=1, stride=stride, bias=False),
                nn.BatchNorm2d(planes * Bottleneck.expansion),
            )
        layers = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * Bottleneck.expansion
        layers += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    # ------------------------------------------------------------------ paths
    def _native_ok(self, x: torch.Tensor) -> bool:
        if not (self.fused and x.is_cuda and x.dim() == 4):
            return False
        return all(m.affine and m.track_running_stats for m in self.modules()
                   if isinstance(m, nn.modules.batchnorm._BatchNorm))

    def _forward_torch(self, x: torch.Tensor) -> torch.Tensor:
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))

    def _forward_native(self, x: torch.Tensor) -> torch.Tensor:
        from ..ops.bn_nhwc import bn_act, global_avg_pool, max_pool_3x3s2

        cdtype = compute_dtype(x) if self.amp_dtype is not None else torch.float32
        _PACKS.clear()
        # the weight-gradient reductions of this step's backward in one launch, unless a DDP
        # reducer (or a peer rank) may read gradients while the backward still runs
        _igemm.WgradBatch.active = (torch.is_grad_enabled() and not getattr(self, "_dpa_ddp_wrapped", False)
                                    and not _multi_rank())
        if _igemm.ENABLED and cdtype in (torch.bfloat16, torch.float16):
            # every implicit-GEMM conv's filters for this step in one launch (with the flipped
            # transpose where the data gradient runs on the kernels: every 3x3, and the 1x1
            # convs ops/conv_igemm.dgrad_1x1_here selects -- all of them by default)
            pack = getattr(self, "_wpack", None)
            if pack is None or pack.cdtype != cdtype:
                convs = [(m, m.kernel_size == (3, 3) or _igemm.dgrad_1x1_here(m.weight.shape[0], 14))
                         for m in self.modules() if isinstance(m, nn.Conv2d) and m.bias is None and m.groups == 1
                         and m.weight.shape[0] % 64 == 0 and m.weight.shape[1] % 64 == 0]
                pack = self._wpack = _igemm.WeightPack(convs, cdtype)
            _PACKS.update(pack.run())
        if _igemm.stem_usable(x, self.conv1, cdtype):
            # 7x7 stem straight from the NCHW image (packed to 4-channel NHWC in-launch)
            c, st = _igemm.stem_conv(x, self.conv1, cdtype, self.bn1)
        else:
            x = x.to(dtype=cdtype, memory_format=torch.channels_last)
            c, st = _conv(x, self.conv1, cdtype, self.bn1)
        x = bn_act(c, self.bn1, relu=True, comm=_comm_of(self.bn1), stats=st)
        x = max_pool_3x3s2(x)
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            bt = None
            for blk in layer:
                x, bt = blk.forward_native(x, cdtype, bt)
        feat = global_avg_pool(x)
        if cdtype in (torch.bfloat16, torch.float16) and os.environ.get("DPA_NATIVE_FC", "1") != "0":
            # fc on the native MFMA linear kernels (ops/head.py: fp32 master weight read
            # in-kernel, fp32 weight / bias gradients) -- no hipBLASLt GEMM left in the step
            from ..ops.head import linear

            return linear(feat, self.fc.weight, self.fc.bias, cdtype)
        return F.linear(feat, self.fc.weight.to(cdtype), self.fc.bias.to(cdtype))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        native = self._native_ok(x)
        fwd = self._forward_native if native else self._forward_torch
        if self.amp_dtype is not None:
            with autocast(dtype=self.amp_dtype, device_type="cuda" if x.is_cuda else "cpu"):
                return fwd(x)
        return fwd(x)


def resnet50(num_classes: int = 1000, amp_dtype: torch.dtype | None = None, fused: bool = True) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes=num_classes, amp_dtype=amp_dtype, fused=fused)
