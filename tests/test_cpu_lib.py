"""CPU-side checks of the native boundary: libgatx.so builds for gfx950, loads, and exports every
entry point include/gatx.h declares, with a ctypes signature for each (no compute calls: there is
no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gatx.h")
LIB = os.path.join(ROOT, "gat-pytorch_amd", "gatx", "libgatx.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gatx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "gatx_edge_forward" in names and "gatx_gemm_f32" in names and len(names) >= 15


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} missing: run `make -C gat-pytorch_amd/csrc` (build())")
    import torch  # noqa: F401  (share torch's HIP runtime, as gatx._lib does)
    return ctypes.CDLL(LIB)


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_binding_covers_header(lib):
    from gatx._lib import SIGNATURES
    assert set(declared_functions()) == set(SIGNATURES)


def _declared_params():
    """{name: [param type strings]} from the header's prototypes."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(gatx_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", src):
        body = " ".join(m.group(2).split())
        out[m.group(1)] = [] if body in ("", "void") else [p.strip() for p in body.split(",")]
    return out


def _ctype_of(decl: str):
    """The ctypes class a header parameter must be bound with."""
    import ctypes as C
    t = decl.rsplit(" ", 1)[0] if " " in decl else decl
    if "*" in decl or "gatx_stream_t" in t:
        return C.c_void_p
    return {"int": C.c_int, "int64_t": C.c_int64, "uint64_t": C.c_uint64, "float": C.c_float,
            "size_t": C.c_size_t, "uint32_t": C.c_uint32}[t.replace("const ", "").strip()]


def test_ctypes_signatures_match_header_prototypes():
    """Every binding has the header's arity and parameter types (an ABI drift here would pass
    garbage pointers to the device)."""
    from gatx._lib import SIGNATURES
    params = _declared_params()
    assert set(params) == set(SIGNATURES)
    for name, decls in params.items():
        got = SIGNATURES[name][1]
        assert len(got) == len(decls), (name, len(got), len(decls))
        for i, (d, g) in enumerate(zip(decls, got)):
            assert _ctype_of(d) is g, (name, i, d, g)


def test_integration_example_matches_header():
    """INTEGRATION.md's hand-written ctypes binding of gatx_edge_forward (what a maintainer would
    copy into the reference) has the header's arity and parameter kinds."""
    import ctypes as C
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"lib\.gatx_edge_forward\.argtypes = (.*?)\n(?!\s)", text, flags=re.S)
    assert m, "INTEGRATION.md lost its gatx_edge_forward binding example"
    got = eval(m.group(1).replace("\\\n", " "), {"ctypes": C})
    want = [_ctype_of(d) for d in _declared_params()["gatx_edge_forward"]]
    assert got == want


def test_library_is_gfx950_code_object():
    data = open(LIB, "rb").read()
    assert b"gfx950" in data


def test_version_and_error_string(lib):
    lib.gatx_version.restype = ctypes.c_int
    lib.gatx_last_error.restype = ctypes.c_char_p
    assert lib.gatx_version() >= 1
    assert isinstance(lib.gatx_last_error(), bytes)


def test_product_has_no_cpu_fallback():
    """The layer refuses CPU tensors instead of silently computing elsewhere."""
    import torch
    from gatx import GATLayer
    layer = GATLayer(4, 3, 2, True, add_self_loops=True)
    with pytest.raises(RuntimeError):
        layer(torch.randn(5, 4), torch.tensor([[0, 1], [1, 2]]))


def test_product_never_imports_oracle():
    """Only tests/, smoke() and bench.py's cpu_baseline leg may use oracle/ (as the checker)."""
    pkg = os.path.join(ROOT, "gat-pytorch_amd")
    pat = re.compile(r"^\s*(from\s+oracle|import\s+oracle)|gat_oracle", re.M)
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(dp, f)).read()
                assert not pat.search(text.replace("oracle/gat_oracle.py", "")), f
