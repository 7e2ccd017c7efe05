"""The C-ABI library: builds for gfx950, loads, and exports exactly what include/rag_retrieval.h declares.
No compute calls (no GPU here)."""
import os
import sys
import re
import subprocess

import pytest

from rag_service_amd import _lib

HEADER = _lib.HEADER_PATH


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rr_[a-z0-9_]+)\s*\(", text)))


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
    exported = set(re.findall(r"\bT (rr_[a-z0-9_]+)\b", out))
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


def test_code_object_targets_gfx950(tmp_path):
    """The library's device code objects are gfx950 ones (llvm-objdump --offloading extracts the bundles next to its
    input: it runs on a copy in tmp_path, so nothing lands in the package directory)."""
    import shutil
    lib_copy = tmp_path / "librag_retrieval.so"
    shutil.copy(_lib.LIB_PATH, lib_copy)
    subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib_copy)], capture_output=True,
                   text=True, cwd=tmp_path)
    bundles = [f.name for f in tmp_path.iterdir() if f.name != lib_copy.name]
    assert any("gfx950" in b for b in bundles), bundles
    assert not any(("gfx9" in b and "gfx950" not in b) for b in bundles), bundles
    assert b"gfx950" in open(_lib.LIB_PATH, "rb").read()


def test_product_path_has_no_oracle_or_fallback():
    pkg = os.path.join(_lib.PKG_ROOT, "rag_service_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert "oracle" not in src.replace("oracle/", ""), f
                assert "import torch" not in src or f in ("dist.py", "batch_processor.py", "serving.py"), f


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_lib.HipRetrievalUnavailable):
        _lib.load_library(str(tmp_path / "nope.so"))


def test_inline_asm_loads_are_hazard_free():
    """Every fused / split-K kernel instantiation: no compiler instruction writes a VGPR that an in-flight
    inline-asm corpus load will still land in, and no VALU result comes out of inline asm (hipcc pads an
    asm output by one wait state; an MFMA operand needs two) — tools/check_asm_loads.py, the hazards of
    cdna_hip_programming.md §5.7 items 1-2. Needs the gfx950 .s from `make isa`."""
    pkg = _lib.PKG_ROOT
    sys.path.insert(0, os.path.join(os.path.dirname(pkg), "tools"))
    from check_asm_loads import check
    # (the split-K kernel's instantiations live in four units, rr_sk_fam_*.hip)
    sk = r"_ZN2rr2sk15sk_score_kernel\w+"
    for unit, pattern, least in (("rr_kernels", r"_ZN2rr18fused_score_kernel\w+", 16), ("rr_sk_fam_exact", sk, 16),
                                 ("rr_sk_fam_s16", sk, 16), ("rr_sk_fam_s8", sk, 16), ("rr_sk_fam_s9", sk, 16)):
        # the library build keeps the assembly (Makefile: -save-temps=obj); rebuild it when it is older than the code
        s_file = os.path.join(pkg, "build", f"{unit}-hip-amdgcn-amd-amdhsa-gfx950.s")
        src = os.path.join(pkg, "csrc", f"{unit}.hip")
        deps = [src, os.path.join(pkg, "csrc", "rr_device.h"), os.path.join(pkg, "csrc", "rr_internal.h"),
                os.path.join(pkg, "csrc", "rr_sk_kernel.h")]
        if not os.path.exists(s_file) or os.path.getmtime(s_file) < max(map(os.path.getmtime, deps)):
            subprocess.check_call(["make", "-C", pkg, "-j8"], stdout=subprocess.DEVNULL)
        text = open(s_file).read()
        syms = re.findall(rf"^({pattern}):", text, flags=re.M)
        assert len(syms) >= least, (unit, len(syms))
        lines = text.split("\n")
        for sym in syms:
            n_asm, bad = check(lines, sym)
            assert not bad, (sym, bad[:5])
