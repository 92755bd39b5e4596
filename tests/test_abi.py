"""C-ABI checks that need no GPU: libdv_hip.so loads, exports exactly the
entry points include/dv_hip.h declares, the ctypes table in _lib.py matches
the header's arity, and every entry point rejects bad arguments on the host
(negative DV_ERR_* code + a dv_last_error message) without touching a device.
"""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dv_hip.h")


@pytest.fixture(scope="module", autouse=True)
def _built_library():
    """Build libdv_hip.so in-tree if this checkout has not built it yet
    (hipcc cross-compiles gfx950 without a GPU)."""
    from dalle2_video import _lib

    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "dalle2-video_amd", "csrc"), "-j8"],
                       check=True, capture_output=True)


def header_decls():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    decls = {}
    for m in re.finditer(r"(?:int|const char\*)\s+(dv_\w+)\s*\(([^)]*)\)\s*;", src):
        params = [p.strip() for p in m.group(2).split(",") if p.strip() and p.strip() != "void"]
        decls[m.group(1)] = params
    return decls


def test_header_parses():
    d = header_decls()
    assert "dv_conv_fwd" in d and "dv_mqa_bwd" in d and "dv_last_error" in d
    assert len(d) >= 30


def test_library_exports_every_declared_symbol():
    from dalle2_video import _lib

    so = _lib.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    declared = set(header_decls())
    assert declared <= exported, f"declared but not exported: {sorted(declared - exported)}"
    ours = {s for s in exported if s.startswith("dv_")}
    assert ours == declared, f"exported but not declared: {sorted(ours - declared)}"


def test_ctypes_table_matches_header():
    from dalle2_video import _lib

    decls = header_decls()
    assert set(_lib.exported_symbols()) == set(decls)
    for name, args in _lib._SIGS.items():
        params = decls[name]
        assert len(args) == len(params), (name, len(args), len(params))
        for a, p in zip(args, params):
            is_ptr = "*" in p
            if is_ptr:
                assert a is ctypes.c_void_p, (name, p)
            elif p.startswith("long long"):
                assert a is ctypes.c_longlong, (name, p)
            elif p.startswith("float"):
                assert a is ctypes.c_float, (name, p)
            else:
                assert p.startswith("int") and a is ctypes.c_int, (name, p)


def test_abi_version_and_error_channel():
    from dalle2_video import _lib

    L = _lib.lib()
    assert L.dv_abi_version() >= 1
    for name, args in _lib._SIGS.items():
        if not args:
            continue
        vals = [None if a is ctypes.c_void_p else a(0) for a in args]
        rc = getattr(L, name)(*vals)
        if name == "dv_gn_path":  # a process-wide mode switch: 0 (automatic) is valid
            assert rc == 0 and L.dv_gn_path(7) == -1
            name = "dv_gn_path"
        else:
            assert rc == -1, (name, rc)  # DV_ERR_INVALID, detected on the host
        msg = L.dv_last_error().decode()
        assert msg.startswith(name + ":"), (name, msg)


def test_call_raises_dverror():
    from dalle2_video import _lib

    with pytest.raises(_lib.DVError, match="dv_gemm_tn_batched"):
        _lib.call("dv_gemm_tn_batched", 1, None, 7, None, 8, None, 32, 1, 8, 8, None)
