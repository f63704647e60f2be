"""ResNet-50 stress model (BASELINE.json config 5) on CPU: torchvision layout,
parameter count, DDP bucket plan vs torch's planner."""
import torch
import torch.distributed as tdist

from ddp_practice_amd.models import resnet50
from ddp_practice_amd.parallel import compute_bucket_assignment


def test_resnet50_layout_and_forward():
    m = resnet50()
    assert sum(p.numel() for p in m.parameters()) == 25_557_032
    sd = m.state_dict()
    assert len(sd) == 320
    for k in ("conv1.weight", "bn1.running_var", "layer1.0.downsample.0.weight", "layer1.0.downsample.1.bias",
              "layer2.3.conv3.weight", "layer3.5.bn2.num_batches_tracked", "layer4.2.bn3.weight", "fc.bias"):
        assert k in sd, k
    assert tuple(sd["layer4.0.conv2.weight"].shape) == (512, 512, 3, 3)
    assert m.layer2[0].conv2.stride == (2, 2) and m.layer2[0].conv1.stride == (1, 1)  # v1.5 stride placement
    out = m(torch.rand(2, 3, 64, 64))
    assert out.shape == (2, 1000)
    out.sum().backward()
    assert all(p.grad is not None for p in m.parameters())


def test_resnet50_bucket_plan_matches_torch():
    """Reverse-order greedy buckets with [1 MiB, 25 MiB] limits: 5 buckets."""
    params = list(resnet50().parameters())
    ours = compute_bucket_assignment(params, 25 * 2 ** 20, 2 ** 20)
    theirs, _ = tdist._compute_bucket_assignment_by_size(params[::-1], [2 ** 20, 25 * 2 ** 20])
    n = len(params)
    assert [sorted(b) for b in ours] == [sorted(n - 1 - i for i in b) for b in theirs]
    sizes = [sum(params[i].numel() * 4 for i in b) / 2 ** 20 for b in ours]
    assert [round(s, 2) for s in sizes] == [7.82, 30.04, 25.04, 25.32, 9.27]


def test_conv1x1_op_matches_conv2d():
    """ops/conv1x1.py (GEMMs on NHWC rows, split-K weight gradient) vs F.conv2d, stride 1 and 2."""
    import torch.nn.functional as F

    from ddp_practice_amd.ops.conv1x1 import conv1x1, wgrad_split

    assert wgrad_split(128 * 56 * 56) == 64 and wgrad_split(128 * 14 * 14) == 8 and wgrad_split(6272) == 2
    assert wgrad_split(1000) == 1
    g = torch.Generator().manual_seed(0)
    for stride in (1, 2):
        x = torch.randn(2, 8, 6, 6, generator=g).contiguous(memory_format=torch.channels_last).requires_grad_()
        w = torch.randn(12, 8, 1, 1, generator=g, requires_grad=True)
        x2 = x.detach().clone().requires_grad_()
        w2 = w.detach().clone().requires_grad_()
        out = conv1x1(x, w, stride, torch.float32)
        ref = F.conv2d(x2, w2, stride=stride)
        assert out.is_contiguous(memory_format=torch.channels_last)
        torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
        gy = torch.randn(ref.shape, generator=g)
        out.backward(gy)
        ref.backward(gy)
        torch.testing.assert_close(x.grad, x2.grad, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(w.grad, w2.grad, rtol=1e-5, atol=1e-5)
        assert w.grad.dtype == torch.float32


def test_conv1x1_grad_tap_accumulates():
    """A tapped residual gradient is accumulated by conv1x1's dgrad GEMM (in place)
    and equals autograd's sum of the two gradient paths."""
    from ddp_practice_amd.ops.conv1x1 import GradTap, conv1x1

    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 8, 5, 5, generator=g).contiguous(memory_format=torch.channels_last).requires_grad_()
    w = torch.randn(6, 8, 1, 1, generator=g)
    gy = torch.randn(2, 6, 5, 5, generator=g)
    extra = torch.randn(2, 8, 5, 5, generator=g).contiguous(memory_format=torch.channels_last)
    tap = GradTap()
    out = conv1x1(x, w, 1, torch.float32, tap)
    tap.grad = extra.clone()  # what the residual BN's backward would have stored
    out.backward(gy)
    x2 = x.detach().clone().requires_grad_()
    (torch.nn.functional.conv2d(x2, w) * gy).sum().backward()
    torch.testing.assert_close(x.grad, x2.grad + extra, rtol=1e-5, atol=1e-5)
    assert tap.grad is None


def test_conv_nhwc_op_matches_conv2d():
    """ops/conv_nhwc.py (fp32 master weight, one cast+layout copy each way) vs F.conv2d."""
    import torch.nn.functional as F

    from ddp_practice_amd.ops.conv_nhwc import conv_nhwc

    g = torch.Generator().manual_seed(3)
    for stride, pad, k in ((1, 1, 3), (2, 1, 3), (2, 3, 7)):
        x = torch.randn(2, 4, 11, 11, generator=g).contiguous(memory_format=torch.channels_last).requires_grad_()
        w = torch.randn(5, 4, k, k, generator=g, requires_grad=True)
        x2, w2 = x.detach().clone().requires_grad_(), w.detach().clone().requires_grad_()
        out = conv_nhwc(x, w, (stride, stride), (pad, pad), torch.float32)
        ref = F.conv2d(x2, w2, stride=stride, padding=pad)
        assert out.is_contiguous(memory_format=torch.channels_last)
        torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
        gy = torch.randn(ref.shape, generator=g)
        out.backward(gy)
        ref.backward(gy)
        torch.testing.assert_close(x.grad, x2.grad, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(w.grad, w2.grad, rtol=1e-4, atol=1e-4)
        assert w.grad.is_contiguous() and w.grad.dtype == torch.float32
