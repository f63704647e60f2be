"""Loader for the native extension ``ddp_practice_amd._C``.

Policy: on a machine with a HIP device the extension is REQUIRED — every op
that has a native kernel raises if ``_C`` cannot be imported (no silent eager
fallback).  On a CPU-only host (``torch.cuda.is_available()`` is False) the
package still imports and the pure-PyTorch reference paths run, which is what
the CPU test tier and the ``origin_main.py`` plumbing config use.
"""
from __future__ import annotations

import hashlib
import importlib
import importlib.util
import os
import sys
import warnings
from pathlib import Path

_C = None
_ERR: Exception | None = None
CSRC = Path(__file__).resolve().parent / "csrc"


def source_digest(csrc: Path = CSRC) -> str:
    """sha1 over every native source (relative path + bytes, sorted): the value build.py
    compiles into ``_C.so`` as ``_C.source_digest``."""
    h = hashlib.sha1()
    for f in sorted(p for p in Path(csrc).rglob("*") if p.suffix in (".hip", ".cpp", ".h") and p.is_file()):
        h.update(f.relative_to(csrc).as_posix().encode())
        h.update(b"\0")
        h.update(f.read_bytes())
    return h.hexdigest()


class StaleExtensionError(RuntimeError):
    pass


def check_fresh(built: str | None, csrc: Path = CSRC, strict: bool | None = None) -> bool:
    """Compare the loaded extension's source digest with the sources in the tree.

    A GPU run after an un-rebuilt source edit would otherwise test the old kernels and
    still report green (Weak 8).  ``strict`` (default: a HIP device is present,
    or DPA_STRICT_EXT=1) raises :class:`StaleExtensionError`; otherwise warns.
    DPA_ALLOW_STALE_EXT=1 skips the check.  Returns True when fresh (or unverifiable:
    no sources shipped next to the package)."""
    if os.environ.get("DPA_ALLOW_STALE_EXT") == "1" or not Path(csrc).is_dir():
        return True
    tree = source_digest(csrc)
    if built == tree:
        return True
    if strict is None:
        import torch

        strict = os.environ.get("DPA_STRICT_EXT") == "1" or torch.cuda.is_available()
    msg = (f"ddp_practice_amd native extension is stale: built from sources {built or '<no digest>'}, "
           f"tree is {tree}. Run `python -m ddp_practice_amd.build` (DPA_ALLOW_STALE_EXT=1 overrides).")
    if strict:
        raise StaleExtensionError(msg)
    warnings.warn(msg, RuntimeWarning, stacklevel=2)
    return False


def load():
    """Import and return the native module, or raise with the build hint."""
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        import torch  # noqa: F401  (loads libamdhip64 / librccl from the torch wheel first)

        so = os.environ.get("DPA_EXT_SO")
        if so:  # experiment build (ddp_practice_amd/build.py DPA_BUILD_TAG), loaded under the same name
            spec = importlib.util.spec_from_file_location("ddp_practice_amd._C", so)
            _C = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_C)
            sys.modules["ddp_practice_amd._C"] = _C
        else:
            _C = importlib.import_module("ddp_practice_amd._C")
    except Exception as e:  # pragma: no cover - exercised only when the build is missing
        _ERR = e
        raise RuntimeError(
            "ddp_practice_amd native extension is not built or failed to load: "
            f"{e!r}. Run `python -m ddp_practice_amd.build`."
        ) from e
    try:
        check_fresh(getattr(_C, "source_digest", None))
    except StaleExtensionError:
        _C = None
        raise
    return _C


def available() -> bool:
    try:
        load()
        return True
    except RuntimeError:
        return False
