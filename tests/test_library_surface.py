"""CPU checks of the C-ABI boundary: libarmi.so builds, loads and exports exactly what
include/armi.h declares, and the ctypes table mirrors it. No compute calls (no GPU here)."""

import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_functions() -> set[str]:
    text = (ROOT / "include" / "armi.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(armi_[a-z0-9_]+)\s*\(", text))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("armi_dense_topk", "armi_sparse_topk", "armi_rrf_fuse", "armi_index_create",
                 "armi_topk_merge_shards", "armi_enc_masked_softmax",
                 "armi_enc_layernorm_residual", "armi_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol(armi_lib):
    missing = [n for n in sorted(declared_functions()) if not hasattr(armi_lib, n)]
    assert not missing, missing


def test_ctypes_table_matches_header(armi_lib):
    from audio_rag_amd import _armi

    assert set(_armi.SIGNATURES) == declared_functions()


def test_abi_version_and_error_path(armi_lib):
    from audio_rag_amd import _armi

    assert armi_lib.armi_abi_version() == _armi.ABI_VERSION
    # argument validation runs before any device work: a null index must fail cleanly
    with pytest.raises(_armi.ArmiError, match="index is null"):
        _armi.call("armi_dense_topk", None, None, 1, 5, None, None, None, None, None, None, None,
                   0, None)
    with pytest.raises(_armi.ArmiError, match="list widths"):
        _armi.call("armi_rrf_fuse", None, None, 0, None, None, 1, 1, 2, 5, None, None, None, None)


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    from audio_rag_amd import _armi

    monkeypatch.setattr(_armi, "_lib", None)
    with pytest.raises(_armi.ArmiUnavailable):
        _armi.load(tmp_path / "libarmi.so")
