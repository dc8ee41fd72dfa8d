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


def test_gemm_describe_names_the_dispatched_kernel():
    """ltx_gemm_describe (host-only: the dispatcher's plan, no launch) names the kernel rocprof
    reports for the config-A shapes, which is what bench.py's roofline attributes timings to."""
    import ctypes
    from ltx_amd import _lib
    lib = _lib.load()

    def name(M, N, K, K2=0, epi="store", rank=0):
        buf = ctypes.create_string_buffer(256)
        assert lib.ltx_gemm_describe(M, N, K, K2, _lib.EPI[epi], rank, None, buf, 256) == 0
        return buf.value.decode()
    M = 8 * 1792
    # N = 2048 tiles: 64 x 8 = 512 of 224 rows fill two rounds exactly; the ring kernel by default
    assert name(M, 2048, 8192) == "ltx::gemm_ring_kernel<0, 0, 7, 0>(ltx::GemmParams)"
    assert name(M, 8192, 2048, epi="gelu") == "ltx::gemm_ring_kernel<1, 0, 8, 0>(ltx::GemmParams)"
    assert name(M, 2048, 2048, K2=64) == "ltx::gemm_ring_kernel<0, 0, 7, 1>(ltx::GemmParams)"
    # K % 128 != 0 keeps gemm_nt_kernel_t; variant 15 selects it everywhere
    assert name(M, 2048, 2112) == "ltx::gemm_nt_kernel_t<0, 0, 224, 4, 0>(ltx::GemmParams)"
    assert lib.ltx_gemm_set_variant(15) == 0
    try:
        assert name(M, 2048, 8192) == "ltx::gemm_nt_kernel_t<0, 0, 224, 4, 0>(ltx::GemmParams)"
        assert name(M, 8192, 2048, epi="gelu") == "ltx::gemm_nt_kernel_t<1, 0, 256, 8, 0>(ltx::GemmParams)"
    finally:
        lib.ltx_gemm_set_variant(0)
    # the text side (M = 256 rows) runs the 128x128 kernel with three LDS stages
    assert name(256, 4096, 2048, K2=128).startswith("ltx::gemm_nt_kernel<0, 0, 3>")


def test_gemm_set_variant_rejects_removed_schedules():
    """Only the kernel / tile-height knobs remain (0 / 13 / 14 / 15 / 20); the not-adopted
    schedules are no longer in the library (tools/experiments/)."""
    from ltx_amd import _lib
    lib = _lib.load()
    assert lib.ltx_gemm_set_variant(13) == 0
    assert lib.ltx_gemm_set_variant(0) == 0
    assert lib.ltx_gemm_set_variant(15) == 0
    assert lib.ltx_gemm_set_variant(20) == 0
    for v in (21, 22, 30, 40, 50, 60):
        assert lib.ltx_gemm_set_variant(v) != 0
    assert lib.ltx_gemm_set_variant(0) == 0


def test_bench_traffic_lookup_reads_newest_profile():
    """bench.py's roofline.traffic comes from the newest committed profiles/r*_traffic.json, with
    kernel names compared after dropping the argument list and trailing default (0) template
    arguments, and names the file it used."""
    import glob
    import importlib.util
    import json
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(repo, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench._kernel_key("void ltx::gemm_nt_kernel_t<0, 0, 224, 4, 0>(ltx::GemmParams)") == \
        "ltx::gemm_nt_kernel_t<0,0,224,4>"
    newest = sorted(glob.glob(os.path.join(repo, "profiles", "r*_traffic.json")))[-1]
    table = json.load(open(newest))["bytes_per_launch"]
    name, val = max(((k, v) for k, v in table.items() if k.startswith("ltx::gemm_")),
                    key=lambda kv: kv[1])
    got, src = bench.load_traffic(name + "(ltx::GemmParams)")
    assert src == os.path.basename(newest) and got == val
    got, why = bench.load_traffic("ltx::no_such_kernel<1>")
    assert got is None and "no entry" in why
