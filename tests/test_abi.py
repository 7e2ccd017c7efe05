"""The C-ABI library: builds for gfx950, loads, and exports exactly what include/rag_retrieval.h declares.
No compute calls (no GPU here)."""
import os
import re
import subprocess

import pytest

from rag_service_amd import _lib

HEADER = _lib.HEADER_PATH


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rr_[a-z_]+)\s*\(", text)))


def header_defines():
    out = {}
    for m in re.finditer(r"#define\s+(RR_[A-Z0-9_]+)\s+(-?\d+)", open(HEADER).read()):
        out[m.group(1)] = int(m.group(2))
    return out


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.load_library()


def test_library_exports_every_header_symbol(lib):
    fns = header_functions()
    assert len(fns) >= 20
    for name in fns:
        assert hasattr(lib, name), name
    assert set(fns) == set(_lib.SIGNATURES), set(fns) ^ set(_lib.SIGNATURES)


def test_exported_dynamic_symbols_match(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (rr_[a-z_]+)\b", out))
    assert exported == set(header_functions())


def test_constants_match_header():
    defs = header_defines()
    for name, val in defs.items():
        if hasattr(_lib, name):
            assert getattr(_lib, name) == val, name
    assert defs["RR_ABI_VERSION"] == _lib.RR_ABI_VERSION


def test_version_and_error_string_without_gpu(lib):
    assert lib.rr_abi_version() == _lib.RR_ABI_VERSION
    assert isinstance(lib.rr_last_error(), bytes)


def test_code_object_targets_gfx950():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", _lib.LIB_PATH, "-d", "--section=none"],
                         capture_output=True, text=True)
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_product_path_has_no_oracle_or_fallback():
    pkg = os.path.join(_lib.PKG_ROOT, "rag_service_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert "oracle" not in src.replace("oracle/", ""), f
                assert "import torch" not in src or f == "dist.py" or f == "batch_processor.py", f


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_lib.HipRetrievalUnavailable):
        _lib.load_library(str(tmp_path / "nope.so"))
