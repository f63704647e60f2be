"""In-tree build of the native extension ``ddp_practice_amd/_C.so``.

One explicit hipcc command per translation unit (gfx950 only), compiled in
parallel, then one link step.  No hipify, no setuptools/JIT machinery: the
resulting ``.so`` lives inside the package so it travels with the repo to the
GPU box and is the file ``import ddp_practice_amd._C`` loads.

The extension links against the HIP runtime and RCCL that ship inside the
PyTorch wheel (same SONAMEs ``libamdhip64.so.7`` / ``librccl.so.1`` as
``/opt/rocm``), so the process has exactly one HIP runtime and one RCCL.

Usage:  python -m ddp_practice_amd.build [-j N] [--force]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
# experiment builds: DPA_BUILD_TAG=x [DPA_EXTRA_CFLAGS="-DFOO"] -> ddp_practice_amd/_C_x.so
# (load it with DPA_EXT_SO=ddp_practice_amd/_C_x.so); the default build is untouched
# DPA_SANITIZE=1: host code under AddressSanitizer + UBSan (device code untouched), built
# as ddp_practice_amd/_C_asan.so and run on the CPU by scripts/asan_check.sh
_SANITIZE = os.environ.get("DPA_SANITIZE", "0") == "1"
_TAG = os.environ.get("DPA_BUILD_TAG", "asan" if _SANITIZE else "")
BUILD = PKG.parent / "build" / ("native" + (f"_{_TAG}" if _TAG else ""))
TARGET = PKG / (f"_C_{_TAG}.so" if _TAG else "_C.so")
ARCH = "gfx950"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_dirs():
    import torch  # noqa: F401  (only for paths)
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths("cuda")
    lib = ce.library_paths("cuda")
    return inc, lib


def sources() -> list[Path]:
    out = []
    for ext in ("*.hip", "*.cpp"):
        out += sorted(CSRC.rglob(ext))
    return out


def _flags():
    import torch

    inc, _ = _torch_dirs()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    f = [
        "-std=c++17", "-O3", "-fPIC", f"--offload-arch={ARCH}",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
        "-D__HIP_NO_HALF_OPERATORS__=1", "-D__HIP_NO_HALF_CONVERSIONS__=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-Wno-unused-result", "-Wno-deprecated-declarations",
        "-fno-gpu-rdc", "-munsafe-fp-atomics",
        f"-I{CSRC}", f"-I{sysconfig.get_paths()['include']}",
    ]
    if _SANITIZE:
        # host side only: every -fsanitize= right after -Xarch_host
        for x in ("-fsanitize=address", "-fsanitize=undefined", "-fno-omit-frame-pointer", "-O1", "-g"):
            f += ["-Xarch_host", x]
    f += os.environ.get("DPA_EXTRA_CFLAGS", "").split()
    f += [f"-I{d}" for d in inc]
    return f


def _obj(src: Path) -> Path:
    rel = src.relative_to(CSRC).as_posix().replace("/", "__")
    return BUILD / (rel + ".o")


def _hash_inputs(src: Path, flags: list[str]) -> str:
    h = hashlib.sha1()
    h.update(" ".join(flags).encode())
    h.update(src.read_bytes())
    for hdr in sorted(CSRC.rglob("*.h")):
        h.update(hdr.read_bytes())
    return h.hexdigest()


def _compile(src: Path, flags: list[str], force: bool) -> tuple[Path, bool]:
    obj = _obj(src)
    stamp = obj.with_suffix(".sha1")
    digest = _hash_inputs(src, flags)
    if not force and obj.exists() and stamp.exists() and stamp.read_text() == digest:
        return obj, False
    lang = ["-x", "hip"] if src.suffix in (".hip", ".cpp") else []
    cmd = ["hipcc", *lang, *flags, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    stamp.write_text(digest)
    return obj, True


def build(jobs: int | None = None, force: bool = False, verbose: bool = True) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    flags = _flags()
    srcs = sources()
    jobs = jobs or min(8, os.cpu_count() or 4)
    changed = False
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, s, flags, force) for s in srcs]
        objs = []
        for s, fu in zip(srcs, futs):
            o, c = fu.result()
            objs.append(o)
            changed |= c
            if verbose and c:
                print(f"[build] compiled {s.relative_to(PKG.parent)}", flush=True)
    # the tree's source digest, compiled in as _C.source_digest (checked by _ext.load())
    from ddp_practice_amd._ext import source_digest

    dsrc = BUILD / "source_digest.cpp"
    dtext = f'extern "C" const char dpa_source_digest[] = "{source_digest(CSRC)}";\n'
    dobj = BUILD / "source_digest.o"
    if not dsrc.exists() or dsrc.read_text() != dtext or not dobj.exists():
        dsrc.write_text(dtext)
        r = subprocess.run(["hipcc", "-x", "c++", "-fPIC", "-c", str(dsrc), "-o", str(dobj)],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {dsrc}\n{r.stderr}")
        changed = True
    objs.append(dobj)
    if changed or force or not TARGET.exists():
        _, libdirs = _torch_dirs()
        torch_lib = libdirs[0]
        cmd = ["hipcc", "-shared", "-fPIC", f"--offload-arch={ARCH}", "-fno-gpu-rdc",
               *map(str, objs), "-o", str(TARGET),
               f"-L{torch_lib}", f"-Wl,-rpath,{torch_lib}",
               "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
               "-ltorch_python", "-lamdhip64", "-lrccl",
               # roctx markers (rocprofv3 --marker-trace); ships with the ROCm image
               f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib", "-lrocprofiler-sdk-roctx"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[build] linked {TARGET.relative_to(PKG.parent)}", flush=True)
    return TARGET


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    build(a.j, a.force)


if __name__ == "__main__":
    sys.exit(main())
