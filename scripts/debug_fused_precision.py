"""Per-tensor error of the fused ConvNet op and of torch fp32, both vs float64 (GPU)."""
import copy
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts", 1)[0])
from ddp_practice_amd.models import ConvNet  # noqa: E402
from ddp_practice_amd.ops import convnet_fused  # noqa: E402


def rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


def run(B, dtype):
    torch.manual_seed(0)
    m = ConvNet().cuda()
    with torch.no_grad():
        for bn in (m.layer1[1], m.layer2[1]):
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
            bn.running_mean.uniform_(-0.1, 0.1)
            bn.running_var.uniform_(0.5, 1.5)
    m64, mt = copy.deepcopy(m).double(), copy.deepcopy(m)
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.rand(B, 1, 28, 28, generator=g).cuda()
    go = torch.randn(B, 10, generator=g).cuda()
    acts = {}

    def fwd(mod, xx, tag):
        p1 = mod.layer1(xx)
        p1.retain_grad()
        p2 = mod.layer2(p1)
        p2.retain_grad()
        acts[tag] = (p1, p2)
        return mod.fc(p2.reshape(p2.size(0), -1))

    out = convnet_fused.convnet_forward(m, x, cdtype=dtype)
    r64 = fwd(m64, x.double(), "64")
    rt = fwd(mt, x, "t")
    out.backward(go.to(dtype))
    r64.backward(go.double())
    rt.backward(go)
    print(f"B={B} {dtype}: logits ours {rel(out, r64):.2e} torch {rel(rt, r64):.2e}")
    for (n, p), (_, q), (_, t) in zip(m.named_parameters(), m64.named_parameters(), mt.named_parameters()):
        print(f"  {n:18s} ours {rel(p.grad, q.grad):.2e}  torch {rel(t.grad, q.grad):.2e}  |g|={q.grad.norm():.3e}")
    for bn, bnr, bnt, nm in ((m.layer1[1], m64.layer1[1], mt.layer1[1], "bn1"),
                             (m.layer2[1], m64.layer2[1], mt.layer2[1], "bn2")):
        print(f"  {nm} running_var ours {rel(bn.running_var, bnr.running_var):.2e} "
              f"torch {rel(bnt.running_var, bnr.running_var):.2e}")


if __name__ == "__main__":
    for B in (32, 100):
        run(B, torch.float32)
