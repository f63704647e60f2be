"""Does the package's SGD (multi-tensor launch, and the fused plain launch) round exactly as
torch.optim.SGD's foreach implementation on this device?  Prints the largest parameter /
momentum-buffer difference after a few steps for several hyper-parameter sets.
    python scripts/exp/sgd_torch_bitwise.py"""
import sys

import torch

sys.path.insert(0, ".")


def run(opt_cls, kw, shapes, steps, fused=None, seed=0):
    from ddp_practice_amd.optim import sgd as sgd_mod

    if fused is not None:
        sgd_mod._PLAIN_FUSED = fused
    g = torch.Generator(device="cpu").manual_seed(seed)
    ps = [torch.randn(s, generator=g).cuda().requires_grad_() for s in shapes]
    opt = opt_cls(ps, **kw)
    for i in range(steps):
        for p in ps:
            p.grad = torch.randn(p.shape, generator=g).cuda()
        opt.step()
    torch.cuda.synchronize()
    return [p.detach().clone() for p in ps], [opt.state[p].get("momentum_buffer") for p in ps]


def main():
    from ddp_practice_amd.optim import SGD

    shapes = [(400,), (16,), (32, 16, 5, 5), (10, 1568), (7,), (4099,)]
    cfgs = [dict(lr=0.05, momentum=0.9), dict(lr=0.1, momentum=0.9, weight_decay=5e-4),
            dict(lr=0.1, momentum=0.9, dampening=0.1, nesterov=False), dict(lr=0.1, momentum=0.9, nesterov=True,
                                                                            weight_decay=1e-4),
            dict(lr=0.01), dict(lr=0.05, momentum=0.9, maximize=True)]
    for kw in cfgs:
        ref_p, ref_b = run(lambda ps, **k: torch.optim.SGD(ps, foreach=True, **k), kw, shapes, 4)
        for name, fused in (("multi-tensor", False), ("fused-plain", True)):
            p, b = run(SGD, kw, shapes, 4, fused=fused)
            dp = max((x - y).abs().max().item() for x, y in zip(p, ref_p))
            db = max(((x - y).abs().max().item() for x, y in zip(b, ref_b) if x is not None and y is not None),
                     default=0.0)
            print(f"{name:13s} {kw}: max |dp| {dp:.3e}  max |dbuf| {db:.3e}", flush=True)


if __name__ == "__main__":
    main()
