"""Does HSA_CU_MASK confine this process's kernels to a CU range?  (runtime/device.shared_cu_mask
gives every rank of a shared-GPU rehearsal 1/W of the CUs.)  A compute-bound bf16 GEMM timed
with the environment as given: with HSA_CU_MASK=0:0-31 on a 256-CU MI355X it should run ~8x
slower than without.
    python scripts/exp/cu_mask_probe.py ; HSA_CU_MASK=0:0-31 python scripts/exp/cu_mask_probe.py"""
import os
import time

import torch


def main():
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        a @ b
    torch.cuda.synchronize()
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        a @ b
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    tf = 2 * 8192 ** 3 / dt / 1e12
    print(f"HSA_CU_MASK={os.environ.get('HSA_CU_MASK')!r}: {dt * 1e3:.2f} ms per 8192^3 bf16 GEMM, {tf:.0f} TF/s",
          flush=True)


if __name__ == "__main__":
    main()
