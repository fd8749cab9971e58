"""The C-ABI library: loads without a GPU, exports every symbol include/msda_hip.h,
include/flat_adamw.h, include/add_layernorm.h, include/ffn_glue.h, include/gemm_small.h,
include/seg_attention.h and include/host_lsa.h declare, and rejects bad arguments with a status + message before
touching a device."""
import ctypes
import os
import re

import pytest

from conftest import PKG, ROOT

HEADERS = [os.path.join(ROOT, "include", h)
           for h in ("msda_hip.h", "flat_adamw.h", "add_layernorm.h", "ffn_glue.h", "gemm_small.h", "seg_attention.h",
                     "host_lsa.h")]


def declared_symbols():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        names |= set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*((?:msda_hip|flat_adamw|mfl)_\w+)\s*\(", text,
                                re.M))
    return sorted(names)


def test_header_symbols_match_binding():
    assert declared_symbols() == sorted(PKG._native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(PKG._native.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_abi_version_and_workspace():
    lib = PKG._native.load_library()
    assert lib.msda_hip_abi_version() == PKG._native.ABI_VERSION
    B, S, M, D, Lq, L, P = 2, 1920, 8, 64, 1920, 4, 4
    # pair-pull backward (16-byte chunks per lane, lists in LDS, any batch size): no workspace;
    # at T = 4096 (S = 7680) the keys alone fill LDS: fp16 stages each (b, m, level) workgroup's
    # entries' (c0, c1) and positions (12 B a sample) in the workspace, bf16 takes the row-block
    # MFMA backward (one int2 row interval per (b, m, level, 32-query tile))
    for dt in (0, 3):
        assert lib.msda_hip_backward_workspace_bytes(dt, B, S, M, D, Lq, L, P) == 0
    # bf16 may take the row-block MFMA backward (the encoder's calls): its tile intervals
    # the row-block path: one int2 interval per (b, m, level, query tile), then the 128-B tail (queue, tile order)
    assert lib.msda_hip_backward_workspace_bytes(2, B, S, M, D, Lq, L, P) == B * M * L * (Lq // 32) * 8 + 128
    assert lib.msda_hip_backward_workspace_bytes(3, 8, 4 * S, M, D, 4 * Lq, L, P) == 8 * M * L * 4 * Lq * P * 12
    assert lib.msda_hip_backward_workspace_bytes(2, 8, 4 * S, M, D, 4 * Lq, L, P) == 8 * M * L * (4 * Lq // 32) * 8 + 128
    # split path (sort + pull): fp64, or heads not made of 16-byte chunks with few workgroups —
    # row table + per-row tap lists
    f64 = lib.msda_hip_backward_workspace_bytes(1, B, S, M, D, Lq, L, P)
    assert f64 >= B * M * S * 8 + B * M * L * 2 * Lq * P * 16
    f32 = lib.msda_hip_backward_workspace_bytes(0, B, S, M, 30, Lq, L, P)
    assert f32 >= B * M * S * 8 + B * M * L * 2 * Lq * P * 8
    assert lib.msda_hip_backward_workspace_bytes(0, 0, S, M, D, Lq, L, P) == 0


@pytest.mark.parametrize("bad", ["levels0", "levels17", "level_overflow", "bad_pad", "bad_dtype", "null_out"])
def test_argument_errors_return_status(bad):
    nat = PKG._native
    lib = nat.load_library()
    shapes, starts, L = [4, 2], [0, 4], 2
    kw = dict(dtype=0, pad=0, S=6, out=ctypes.c_void_p(16), L=L)
    if bad == "levels0":
        kw["L"] = 0
    elif bad == "levels17":
        shapes, starts, kw["L"] = [1] * 17, list(range(17)), 17
        kw["S"] = 17
    elif bad == "level_overflow":
        starts = [0, 5]
    elif bad == "bad_pad":
        kw["pad"] = 7
    elif bad == "bad_dtype":
        kw["dtype"] = 9
    elif bad == "null_out":
        kw["out"] = None
    fake = ctypes.c_void_p(16)  # never dereferenced: validation fails first
    rc = lib.msda_hip_forward(fake, kw["dtype"], nat.host_i64_array(shapes), nat.host_i64_array(starts), kw["L"],
                              fake, fake, kw["out"], 1, kw["S"], 1, 4, 3, 2, kw["pad"], None)
    assert rc == 1
    assert "msda" in nat.last_error()
