"""The C-ABI library builds, loads and exports every symbol include/*.h
declares (no compute calls: this runs without a GPU)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    syms = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        for m in re.finditer(r"^\s*(?:[A-Za-z_][\w\s\*]*?)\b(bpp_\w+)\s*\(", text, flags=re.M):
            syms.add(m.group(1))
    return sorted(syms)


def test_header_declares_api():
    syms = declared_symbols()
    assert "bpp_msm" in syms and "bpp_ctx_create" in syms
    assert len(syms) >= 20


def test_library_exports_every_declared_symbol():
    from bpperm import _lib
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from bpperm import _lib
    missing = [s for s in declared_symbols() if s not in _lib.SIGNATURES]
    assert not missing, missing


def test_no_cpu_fallback_without_library(tmp_path):
    from bpperm import _lib
    with pytest.raises(RuntimeError):
        _lib.load(tmp_path / "missing.so")
