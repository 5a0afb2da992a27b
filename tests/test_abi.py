"""The C-ABI library loads and exports every symbol include/*.h declares; pure
host entry points behave; compute entry points refuse to run without a GPU
(no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if not fn.endswith(".h"):
            continue
        src = open(os.path.join(ROOT, "include", fn)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(rm_\w+)\s*\(", src, re.M):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ("rm_create", "rm_dispatch", "rm_read_rgba8", "rm_read_rgba32f",
                 "rm_get_counters", "rm_last_error", "rm_destroy", "rm_set_float",
                 "rm_camera_look_at", "rm_unshard_rgba8"):
        assert must in names


def test_library_exports_every_declared_symbol(rm):
    lib = rm.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"librm.so lacks {missing}"
    # and the Python mirror binds all of them
    assert set(declared_functions()) <= set(rm.EXPORTED_SYMBOLS)


def test_structs_match_header_sizes(rm):
    # sizes implied by include/rm_api.h (plain C layout, 4-byte fields)
    assert C.sizeof(rm.rm_camera) == 64
    assert C.sizeof(rm.rm_light) == 60
    assert C.sizeof(rm.rm_uniforms) == 64 + 60 + 4 * 5 + 12 + 8 + 4
    assert C.sizeof(rm.rm_counters) == 56
    assert C.sizeof(rm.rm_config) == 36
    assert C.sizeof(rm.rm_camera_state) == 8 + 24 + 48


def test_api_version(rm):
    assert rm.lib().rm_api_version() == 1


def test_argument_validation_without_gpu(rm):
    # invalid configs are rejected before any device call
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(0, 10)
    assert e.value.code == rm.RM_ERR_INVALID
    with pytest.raises(rm.RMError):
        rm.Renderer(16, 16, nshards=2, row_block=0)
    with pytest.raises(rm.RMError):
        rm.sweep_uniforms(0, 120, bounces=6)


def test_no_cpu_fallback(rm):
    if rm.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(16, 16)
    assert e.value.code == rm.RM_ERR_NO_DEVICE
    assert "no HIP device" in str(e.value)
