"""Log every aten fill / zero / zeros / full / copy_ on a CUDA tensor (any dtype) issued
while a hipGraph is being captured, with the Python stack, during a short ConvNet bench run.
Extra arguments go to bench.py, e.g.

  python scripts/exp/find_fill.py --force-collectives     (the DDP + SyncBN step in a world of one)
  python scripts/exp/find_fill.py --amp-dtype fp32
"""
import collections
import runpy
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

seen = collections.Counter()
NAMES = ("fill", "zero", "zeros", "full", "new_zeros", "new_full", "copy_")


class Finder(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.__name__.split(".")[0]
        if name.strip("_") in NAMES or name in NAMES:
            t = out if isinstance(out, torch.Tensor) else (args[0] if args and isinstance(args[0], torch.Tensor) else None)
            if t is not None and t.is_cuda and torch.cuda.is_current_stream_capturing():
                st = "".join(traceback.format_stack(limit=14)[:-1])
                if seen[st] == 0:
                    print(f"=== {func} {t.dtype} shape={tuple(t.shape)}\n{st}", file=sys.stderr, flush=True)
                seen[st] += 1
        return out


sys.argv = ["bench.py", "--steps", "64", "--warmup", "16", "--epochs", "0", "--no-baseline", "--extra-dtypes", "", "--no-steady", *sys.argv[1:]]
with Finder():
    runpy.run_path("bench.py", run_name="__main__")
print("distinct stacks:", len(seen), "calls:", sum(seen.values()), file=sys.stderr)
