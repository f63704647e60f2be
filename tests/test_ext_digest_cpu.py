"""Stale-binary guard (Weak 8): ``_C.so`` carries the digest of the sources it
was built from and ``_ext.load()`` refuses (on a HIP host) a binary whose digest differs
from the tree, so a GPU run after an un-rebuilt source edit cannot test old kernels."""
import shutil
import warnings

import pytest

from ddp_practice_amd import _ext


def test_editing_a_hip_file_without_rebuilding_is_an_error(tmp_path):
    csrc = tmp_path / "csrc"
    shutil.copytree(_ext.CSRC, csrc)
    built = _ext.source_digest(csrc)
    assert _ext.check_fresh(built, csrc, strict=True)
    hip = sorted(csrc.rglob("*.hip"))[0]
    hip.write_text(hip.read_text() + "\n// edited\n")
    with pytest.raises(_ext.StaleExtensionError, match="stale"):
        _ext.check_fresh(built, csrc, strict=True)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert not _ext.check_fresh(built, csrc, strict=False)
    assert any("stale" in str(x.message) for x in w)


def test_header_edit_and_new_file_change_the_digest(tmp_path):
    csrc = tmp_path / "csrc"
    shutil.copytree(_ext.CSRC, csrc)
    d0 = _ext.source_digest(csrc)
    (csrc / "common.h").write_text((csrc / "common.h").read_text() + " ")
    d1 = _ext.source_digest(csrc)
    (csrc / "kernels" / "new.hip").write_text("")
    assert len({d0, d1, _ext.source_digest(csrc)}) == 3


def test_missing_digest_is_stale(tmp_path):
    with pytest.raises(_ext.StaleExtensionError):
        _ext.check_fresh(None, _ext.CSRC, strict=True)


def test_in_tree_extension_matches_tree():
    """The built ``_C.so`` (when present) was built from the current sources."""
    so = _ext.CSRC.parent / "_C.so"
    if not so.exists():
        pytest.skip("extension not built")
    C = _ext.load()
    assert C.source_digest == _ext.source_digest()
