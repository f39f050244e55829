"""CPU tests of the C-ABI library: it loads, exports every function include/*.h declares, reports a
missing GPU loudly (no CPU fallback), and the host-side mirror rejects misuse without a device."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in ("gwaoi.h", "gwaoi_tools.h", "gwaoi_strips.h", "gwaoi_sync.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_ ]*[\s\*]+(gwaoi_[a-z0-9_]+)\s*\(", src, re.M):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_boundary():
    names = declared_functions()
    for n in ("gwaoi_create", "gwaoi_enter", "gwaoi_leave", "gwaoi_moved", "gwaoi_stage_moves", "gwaoi_tick",
              "gwaoi_destroy", "gwaoi_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol(gwaoi_lib):
    from goworld_amd import _lib
    names = declared_functions()
    assert set(names) == set(_lib.ABI_SYMBOLS) | set(_lib.TOOL_SYMBOLS) | set(_lib.STRIP_SYMBOLS) | set(_lib.SYNC_SYMBOLS)
    for n in names:
        assert hasattr(gwaoi_lib, n), n
        assert ctypes.cast(getattr(gwaoi_lib, n), ctypes.c_void_p).value


def test_library_has_gfx950_code_object():
    from goworld_amd import _lib
    blob = open(_lib.SO_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"k_sweep" in blob  # the hand-written sweep kernel is in the bundle


def test_no_gpu_fails_loudly(gwaoi_lib):
    from goworld_amd import _lib
    from goworld_amd.engine import Engine
    if _lib.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.GwaoiError) as e:
        Engine(100.0, 1024)
    assert e.value.code == _lib.GWAOI_ERR_HIP
    assert b"no HIP device" in gwaoi_lib.gwaoi_last_error()


def test_invalid_arguments(gwaoi_lib):
    from goworld_amd import _lib
    h = ctypes.c_void_p()
    assert gwaoi_lib.gwaoi_create(0.0, 16, 0, ctypes.byref(h)) == _lib.GWAOI_ERR_INVALID   # dist <= 0
    assert gwaoi_lib.gwaoi_create(-1.0, 16, 0, ctypes.byref(h)) == _lib.GWAOI_ERR_INVALID
    assert gwaoi_lib.gwaoi_create(100.0, 0, 0, ctypes.byref(h)) == _lib.GWAOI_ERR_INVALID  # capacity 0
    assert gwaoi_lib.gwaoi_enter(None, 0, 0.0, 0.0) == _lib.GWAOI_ERR_INVALID
    assert gwaoi_lib.gwaoi_tick(None, None) == _lib.GWAOI_ERR_INVALID
    assert gwaoi_lib.gwaoi_destroy(None) == _lib.GWAOI_OK
    assert gwaoi_lib.gwaoi_version().startswith(b"gwaoi")


def test_product_does_not_import_oracle():
    """The product path never reaches the oracle (it is test infrastructure only)."""
    for dirpath, _, files in os.walk(os.path.join(ROOT, "goworld_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in src.replace("oracle/", "").lower() or f == "__init__.py", f
