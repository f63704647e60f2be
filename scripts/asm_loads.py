"""ISA audit of a kernel's memory round trips (how this round's ConvNet latency cuts were found).

    python scripts/asm_loads.py KERNEL_SUBSTRING [SRC.hip] [N]

compiles SRC (default csrc/kernels/convnet_fused.hip) for gfx950 with the extension's
flags (`hipcc --cuda-device-only -S`) and prints, for the first kernel whose mangled name
contains KERNEL_SUBSTRING, the ordered sequence of global / buffer / LDS-DMA loads,
`s_waitcnt vmcnt`, barriers, atomics and stores.  What to look for:
  * a `global_load_ushort` from the kernarg segment followed by `vmcnt(0)` -- blockDim /
    gridDim read mid-kernel (a hidden-argument load whose wait retires every earlier load);
  * a load inside its own basic block followed by `vmcnt(0)` -- a conditional load hipcc
    branched around (make it unconditional: clamped index, masked value);
  * `vmcnt(0)` at a loop header ahead of a batch of loads (peel the first iteration).
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    if len(sys.argv) < 2:
        print(__doc__)
        return 2
    pat = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "ddp_practice_amd/csrc/kernels/convnet_fused.hip")
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    from ddp_practice_amd import build as b

    out = "/tmp/_asm_loads.s"
    cmd = ["hipcc", "-x", "hip", *b._flags(), "--cuda-device-only", "-S", src, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        print(r.stderr)
        return r.returncode
    s = open(out).read()
    for f in re.split(r"\n(?=_Z\S*: ;)", s):
        name = f.split(":", 1)[0]
        if pat in name:
            print(name)
            k = 0
            for i, line in enumerate(f.splitlines()):
                t = line.strip()
                if re.match(r"(global_load|buffer_load|s_waitcnt vmcnt|s_barrier|global_atomic|global_store|s_sleep)", t):
                    print(f"{i:6d}  {t[:90]}")
                    k += 1
                    if k >= n:
                        break
            return 0
    print(f"no kernel matching {pat!r} in {src}")
    return 1


if __name__ == "__main__":
    sys.exit(main())
