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
    assert C.sizeof(rm.rm_config) == 64  # struct_size + magic + 12 int32 + the devices pointer
    assert C.sizeof(rm.rm_camera_state) == 8 + 24 + 48


def test_struct_layouts_match_the_c_compiler(rm, tmp_path):
    """Every field offset of the ctypes mirrors equals the C compiler's for
    include/rm_api.h (catches a field added on one side only)."""
    import subprocess
    structs = {"rm_config": rm.rm_config, "rm_uniforms": rm.rm_uniforms,
               "rm_counters": rm.rm_counters, "rm_primitive": rm.rm_primitive,
               "rm_camera_state": rm.rm_camera_state, "rm_input_state": rm.rm_input_state}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rm_api.h"', "int main(void) {"]
    for name, py in structs.items():
        lines.append(f'printf("{name} size %zu\\n", sizeof({name}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{name} {f} %zu\\n", offsetof({name}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l}
    for name, py in structs.items():
        assert got[(name, "size")] == C.sizeof(py), name
        for f, _ in py._fields_:
            assert got[(name, f)] == getattr(py, f).offset, (name, f)


def test_api_version(rm):
    assert rm.lib().rm_api_version() == 6 == rm.RM_API_VERSION


def test_config_struct_size_is_checked(rm):
    """a host built against an older rm_api.h passes a smaller
    rm_config without struct_size (its first word is the width); rm_create
    refuses it before reading any later field."""
    cfg = rm.rm_config()
    assert rm.lib().rm_config_init(C.byref(cfg), 64, 32) == 0
    assert (cfg.struct_size, cfg.magic, cfg.width, cfg.height, cfg.device, cfg.outputs, cfg.nshards,
            cfg.ngpus) == (C.sizeof(rm.rm_config), rm.RM_CONFIG_MAGIC, 64, 32, -1, rm.RM_OUT_RGBA8, 1, 0)
    old = rm.rm_config(struct_size=3840, magic=2160)  # a v1/v2 layout (width, height) read as v4
    h = C.c_void_p()
    assert rm.lib().rm_create(C.byref(h), C.byref(old)) == rm.RM_ERR_INVALID
    assert b"struct_size" in rm.lib().rm_last_error(None)
    assert not h.value
    # a v3 host's struct has the same size as v4's (56 on LP64) and its
    # second word is the width: the magic refuses it
    v3 = rm.rm_config(struct_size=C.sizeof(rm.rm_config), magic=1920, width=1080)
    assert rm.lib().rm_create(C.byref(h), C.byref(v3)) == rm.RM_ERR_INVALID
    assert b"magic" in rm.lib().rm_last_error(None)
    assert not h.value
    # a v4 host (magic "RMC4", 56 bytes, no rank0_rows) is refused by size and magic
    v4 = rm.rm_config(struct_size=56, magic=0x34434D52, width=64, height=32)
    assert rm.lib().rm_create(C.byref(h), C.byref(v4)) == rm.RM_ERR_INVALID
    v4.struct_size = C.sizeof(rm.rm_config)
    assert rm.lib().rm_create(C.byref(h), C.byref(v4)) == rm.RM_ERR_INVALID
    assert b"magic" in rm.lib().rm_last_error(None)
    assert not h.value
    # a v5 host (magic "RMC5"): the same 64 bytes as v6, whose shard_format sits where
    # v5 had ngpus: refused by the magic
    v5 = rm.rm_config(struct_size=C.sizeof(rm.rm_config), magic=0x35434D52, width=64, height=32)
    assert rm.lib().rm_create(C.byref(h), C.byref(v5)) == rm.RM_ERR_INVALID
    assert b"magic" in rm.lib().rm_last_error(None)
    assert not h.value


def test_shard_format_validation_without_gpu(rm):
    """rm_config.shard_format (API version 6) outside RM_SHARD_* is refused before any
    device call, for one-device and multi-GPU contexts alike."""
    for kw in (dict(nshards=2, row_block=8), dict(ngpus=2)):
        for bad in (-1, 3):
            with pytest.raises(rm.RMError) as e:
                rm.Renderer(64, 64, shard_format=bad, **kw)
            assert e.value.code == rm.RM_ERR_INVALID and "shard_format" in str(e.value)


def _model_owner(H, R, R0, N):
    """Independent model of the weighted interleave: the owner shard and local row
    of every global row, walking the rounds."""
    own, loc, cnt = [], [], [0] * N
    while len(own) < H:
        for s in range(N):
            for _ in range(R0 if s == 0 else R):
                own.append(s)
                loc.append(cnt[s])
                cnt[s] += 1
    return own[:H], loc[:H]


@pytest.mark.parametrize("H,R,R0,N", [(2160, 8, 7, 8), (2160, 8, 0, 4), (541, 3, 2, 5), (64, 8, 13, 2),
                                      (17, 4, 1, 3), (100, 8, 8, 1)])
def test_every_shard_function_against_the_model(rm, H, R, R0, N):
    """every shard function of the C-ABI, called directly with a
    weighted map, agrees with the pure model; all take (height, row_block,
    rank0_rows, nshards, ...) in that order (API version 6)."""
    L = rm.lib()
    r0 = R0 or R
    own, loc = _model_owner(H, R, r0, max(N, 1))
    n, cap = C.c_int32(0), C.c_int32(0)
    caps = set()
    for s in range(N):
        assert L.rm_shard_rows(H, R, R0, N, s, C.byref(n), C.byref(cap)) == rm.RM_OK
        caps.add(cap.value)
        mine = [y for y in range(H) if own[y] == s]
        assert n.value == len(mine)
        for j, y in enumerate(mine):
            assert L.rm_shard_to_global(H, R, R0, N, s, j) == y
        for j in range(len(mine), cap.value):
            assert L.rm_shard_to_global(H, R, R0, N, s, j) == -1
    assert len(caps) == 1, "every shard image has the same rows_cap"
    for y in range(H):
        s_, l_ = C.c_int32(-1), C.c_int32(-1)
        assert L.rm_shard_owner(H, R, R0, N, y, C.byref(s_), C.byref(l_)) == rm.RM_OK
        assert (s_.value, l_.value) == (own[y], loc[y])
    # the v5 signature's order (shard before nshards) no longer binds
    assert not hasattr(L, "rm_shard_row") and not hasattr(L, "rm_shard_rows_cap")
    assert not hasattr(L, "rm_shard_global_row")


def test_multi_gpu_config_validation_without_gpu(rm):
    # RCCL-gathered frames are RGBA8 / RGBA32F, without counters; rejected before any device call
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(64, 64, ngpus=2, outputs=4)
    assert e.value.code == rm.RM_ERR_INVALID
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(64, 64, ngpus=2, counters=True)
    assert e.value.code == rm.RM_ERR_INVALID
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(64, 64, ngpus=2, nshards=2, row_block=8)
    assert e.value.code == rm.RM_ERR_INVALID
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(64, 64, ngpus=-1)
    assert e.value.code == rm.RM_ERR_INVALID


def test_comm_unique_id_without_gpu(rm):
    """ncclGetUniqueId needs no device: rank 0 of a host without GPUs (a launcher)
    can make the id; two calls give different ids."""
    a, b = rm.comm_unique_id(), rm.comm_unique_id()
    assert len(a) == rm.COMM_ID_BYTES and a != b


def test_argument_validation_without_gpu(rm):
    # invalid configs are rejected before any device call
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(0, 10)
    assert e.value.code == rm.RM_ERR_INVALID
    with pytest.raises(rm.RMError):
        rm.Renderer(16, 16, nshards=2, row_block=0)
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(16, 16, nshards=2, row_block=8, rank0_rows=-1)
    assert e.value.code == rm.RM_ERR_INVALID
    with pytest.raises(rm.RMError):
        rm.sweep_uniforms(0, 120, bounces=6)


def test_no_cpu_fallback(rm):
    if rm.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(rm.RMError) as e:
        rm.Renderer(16, 16)
    assert e.value.code == rm.RM_ERR_NO_DEVICE
    assert "no HIP device" in str(e.value)
