"""Per-key differences between fp32 ConvNet training with and without the slab sink (the
fused plain-SGD launch), eagerly and graph-replayed -- the quantities
tests/test_convnet_fused_gpu.py::test_fp32_plain_fused_step_with_slab_sink compares, printed
whole, to localise a mismatch.
    python scripts/exp/fp32_sink_diff.py [eager_steps] [graph_runs]"""
import copy
import sys

import torch

sys.path.insert(0, ".")
from tests.test_convnet_fused_gpu import _model  # noqa: E402


def run(fused, eager_steps, graph_runs, defer=True):
    from ddp_practice_amd.data import DeviceLoader, synthetic
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD, sgd as sgd_mod
    from ddp_practice_amd.runtime import CapturedStep

    sgd_mod._PLAIN_FUSED = fused
    ds = synthetic(32 * 12, seed=5)
    m = _model()
    loader = DeviceLoader(ds, batch_size=32, shuffle=False, device="cuda", dtype=torch.float32)
    images, labels = loader.static_batch()
    opt, crit = SGD(m.parameters(), lr=0.05, momentum=0.9), CrossEntropyLoss()
    if fused:
        assert m.set_slab_sink(opt)

    def step():
        loader.fill_(images, labels, defer=defer)
        loss = crit(m(images), labels)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    loader.start_epoch()
    for _ in range(eager_steps):
        step()
    if graph_runs:
        runner = CapturedStep(step, warmup=1, steps_per_graph=2)
        assert runner.capture()
        for _ in range(graph_runs):
            runner.run()
    torch.cuda.synchronize()
    return copy.deepcopy(m.state_dict())


def main():
    eager = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    graph = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    for defer in (True, False):
        a, b, a2 = run(False, eager, graph, defer), run(True, eager, graph, defer), run(False, eager, graph, defer)
        print(f"eager {eager} graph_runs {graph} defer {defer}", flush=True)
        for k in a:
            d = (a[k].float() - b[k].float()).abs().max().item()
            d2 = (a[k].float() - a2[k].float()).abs().max().item()
            print(f"  {k:28s} plain-vs-sink {d:.3e}  plain-vs-plain {d2:.3e}", flush=True)
        if graph:  # each path graph-replayed vs the same number of eager steps (CapturedStep runs one
            # warm-up step eagerly first)
            for fused, g in ((False, a), (True, b)):
                e = run(fused, eager + 1 + 2 * graph, 0, defer)
                worst = max(((g[k].float() - e[k].float()).abs().max().item(), k) for k in g)
                print(f"  {'sink' if fused else 'plain'} graph-vs-eager worst {worst[0]:.3e} ({worst[1]})", flush=True)


if __name__ == "__main__":
    main()
