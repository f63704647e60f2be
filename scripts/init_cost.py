"""Where the first ~1.5 s of a CLI run goes on the GPU box: HIP init, native extension
load, first launches (prints one line per stage)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
t0 = time.time()
import torch  # noqa: E402

t1 = time.time()
torch.cuda.init()
t2 = time.time()
from ddp_practice_amd import _ext  # noqa: E402

_ext.load()
t3 = time.time()
from ddp_practice_amd.models import ConvNet  # noqa: E402

m = ConvNet(amp_dtype=torch.bfloat16).cuda()
torch.cuda.synchronize()
t4 = time.time()
x = torch.rand(32, 1, 28, 28, device="cuda")
m(x).float().sum().backward()
torch.cuda.synchronize()
t5 = time.time()
m(x).float().sum().backward()
torch.cuda.synchronize()
t6 = time.time()
print(f"import torch {t1 - t0:.3f}s  cuda.init {t2 - t1:.3f}s  ext load {t3 - t2:.3f}s  model.cuda {t4 - t3:.3f}s  "
      f"first fwd+bwd {t5 - t4:.3f}s  second {t6 - t5:.3f}s")
