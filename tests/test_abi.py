"""The C-ABI library loads on the host (no GPU needed) and exports every symbol declared in
include/ltx_hip.h; the Python binding table matches the header. No compute calls here."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ltx_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(ltx_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_entry_points():
    names = header_functions()
    assert "ltx_gemm_bf16_nt" in names and "ltx_attn_fwd" in names and len(names) >= 25


def test_library_exports_every_declared_symbol():
    from ltx_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} missing: run __graft_entry__.build() first")
    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert set(header_functions()) == set(_lib.exported_symbols())
    assert lib.ltx_abi_version() == 1


def test_ops_refuse_cpu_tensors():
    import torch
    from ltx_amd import ops, _lib
    x = torch.zeros(128, 64, dtype=torch.bfloat16)
    with pytest.raises(_lib.LtxHipError):
        ops.gemm(x, x)
