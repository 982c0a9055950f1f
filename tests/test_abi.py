"""The C-ABI library loads without a GPU and exports exactly what include/gsr.h declares, with the
argument counts the ctypes binding uses (no compute calls: no GPU here)."""
import ctypes
import os
import re

import pytest

from diff_gaussian_rasterization import _C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gsr.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(gsr_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.M | re.S):
        name, args = m.group(1), m.group(2).strip()
        n = 0 if args in ("", "void") else len([a for a in args.split(",") if a.strip()])
        out[name] = n
    return out


def test_header_parses():
    fns = header_functions()
    for required in ("gsr_forward_preprocess", "gsr_num_rendered", "gsr_forward_render", "gsr_backward",
                     "gsr_mark_visible", "gsr_geom_bytes", "gsr_binning_bytes", "gsr_image_bytes",
                     "gsr_backward_bytes", "gsr_version", "gsr_last_error", "gsr_profile_enable",
                     "gsr_profile_read"):
        assert required in fns, required


def test_library_exports_every_declared_symbol():
    lib = _C.load_library()
    for name in header_functions():
        assert hasattr(lib, name), f"{name} declared in gsr.h but not exported"


def test_binding_signatures_match_header():
    fns = header_functions()
    assert set(fns) == set(_C.SIGNATURES), set(fns) ^ set(_C.SIGNATURES)
    for name, nargs in fns.items():
        assert len(_C.SIGNATURES[name][1]) == nargs, f"{name}: header {nargs} args, binding {len(_C.SIGNATURES[name][1])}"


def test_host_only_queries():
    lib = _C.load_library()
    assert lib.gsr_abi_version() == _C.ABI_VERSION
    assert lib.gsr_version().decode().startswith("gsr ")
    assert "gfx950" in lib.gsr_version().decode()
    assert lib.gsr_geom_bytes(1000) >= 1000 * (48 + 8 + 4 * 7)  # records, rect, 7 u32 words
    assert lib.gsr_set_geom_bytes(4, 1000) >= 4 * lib.gsr_geom_bytes(1000) - 4 * 4096
    assert lib.gsr_binning_bytes(5000, 64, 64) >= 5000 * 16
    assert lib.gsr_image_bytes(64, 48) >= 64 * 48 * 8
    assert lib.gsr_backward_bytes(10, 100) >= 100 * 48 + 10 * 13 * 4  # one row per instance + per-Gaussian records
    assert lib.gsr_geom_bytes(0) > 0  # sizes stay valid for P = 0


def test_argument_errors_without_gpu():
    """Argument validation happens before any device work and reports the reference's messages."""
    lib = _C.load_library()
    v = ctypes.c_void_p(16)  # never dereferenced: the call must fail validation first
    rc = lib.gsr_forward_preprocess(10, 0, 1, v, v, 1.0, v, v, v, v, None, v, v, v, 64, 64, 0.5, 0.5, 0,
                                    v, v, None)
    assert rc == 1
    assert b"exactly one of either SHs or precomputed colors" in lib.gsr_last_error()
    rc = lib.gsr_forward_preprocess(10, 0, 1, v, None, 1.0, v, v, v, None, v, v, v, v, 64, 64, 0.5, 0.5, 0,
                                    v, v, None)
    assert rc == 1
    assert b"scale/rotation pair or precomputed 3D covariance" in lib.gsr_last_error()
    assert lib.gsr_forward_render(1, 1, 0, 64, v, v, v, v, v, v, v, None) == 1


def test_oracle_library_builds_and_exports():
    import oracle

    lib = oracle.lib()
    for name in ("oracle_forward_f32", "oracle_forward_f64", "oracle_backward_f32", "oracle_backward_f64",
                 "oracle_eval_sh_f64", "oracle_cov3d_f64"):
        assert hasattr(lib, name)


def test_image_bytes_follow_the_split_decision(monkeypatch):
    """gsr_set_image_bytes_ex sizes the image buffer for the forward's split decision: with the split backward's
    checkpoints (335 MB for one 1024^2 view) only when the forward writes them (one colour set, quadrant waves,
    GSR_BWD_SPLIT not 0); gsr_set_image_bytes stays the upper bound."""
    import ctypes

    lib = _C.load_library()
    K = (ctypes.c_int * 1)(5000)
    full = lib.gsr_set_image_bytes(1, 1024, 1024)
    monkeypatch.delenv("GSR_BWD_SPLIT", raising=False)
    monkeypatch.delenv("GSR_FWD_KERNEL", raising=False)
    split = lib.gsr_set_image_bytes_ex(1, 1000, K, 1024, 1024, 0)
    two = lib.gsr_set_image_bytes_ex(1, 1000, K, 1024, 1024, 1)
    assert split == full and two < full and full - two >= 4096 * 16 * 5 * 256 * 4 - 256
    monkeypatch.setenv("GSR_BWD_SPLIT", "0")
    assert lib.gsr_set_image_bytes_ex(1, 1000, K, 1024, 1024, 0) == two
    K64 = (ctypes.c_int * 64)(*([5000] * 64))
    assert lib.gsr_set_image_bytes_ex(64, 1000, K64, 1024, 1024, 0) == lib.gsr_set_image_bytes(64, 1024, 1024)
