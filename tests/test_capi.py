"""C-ABI boundary: the library loads (no GPU needed) and exports every symbol of
include/autovc_hip.h, and the ctypes table in autovc_amd/_lib.py covers them all."""
import ctypes
import os
import re

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "autovc_hip.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(autovc_[a-z0-9_]+)\s*\(", txt)))


def test_header_has_symbols():
    syms = header_symbols()
    assert "autovc_last_error" in syms and "autovc_stft_mel_f32" in syms


def test_library_exports_header_symbols():
    from autovc_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, f"library lacks {missing}"


def test_ctypes_table_matches_header():
    from autovc_amd import _lib
    assert sorted(_lib.exported_symbols()) == header_symbols()


def test_abi_version_and_error_path():
    from autovc_amd import _lib
    lib = _lib.load()
    assert lib.autovc_abi_version() == 1
    # argument validation runs before any device work: safe without a GPU
    import pytest
    with pytest.raises(ValueError, match="n_utt"):
        _lib.call("autovc_stft_mel_f32", 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0)
