"""Loader for the native extension ``ddp_practice_amd._C``.

Policy: on a machine with a HIP device the extension is REQUIRED — every op
that has a native kernel raises if ``_C`` cannot be imported (no silent eager
fallback).  On a CPU-only host (``torch.cuda.is_available()`` is False) the
package still imports and the pure-PyTorch reference paths run, which is what
the CPU test tier and the ``origin_main.py`` plumbing config use.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys

_C = None
_ERR: Exception | None = None


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
    return _C


def available() -> bool:
    try:
        load()
        return True
    except RuntimeError:
        return False
