"""Runtime scene table, host side: the reference scene as a
table (rm_default_scene, computeShader.glsl:107-123) and the oracle's table mode.

The oracle's table mode evaluates the same GLSL primitives (glsl:83-103) in table
order with opU (glsl:105).  Fed the default table it must reproduce the oracle's
literal transcription of sdf() bit for bit — colours, NaN masks and work counters —
which pins the table semantics (entry order, swizzle, blend, checkers paint, ids,
materials) to the reference scene.  No GPU calls."""
import ctypes as C
import os

import numpy as np
import pytest


def test_default_scene_is_the_reference_scene(rm):
    sc = rm.default_scene()
    assert [p.type for p in sc] == [rm.PRIM_SPHERE, rm.PRIM_SPHERE, rm.PRIM_BLEND, rm.PRIM_TORUS,
                                    rm.PRIM_CAPSULE, rm.PRIM_PLANE]
    assert [p.id for p in sc] == [0, 1, 4, 5, 6, 7]                       # glsl:111-121
    assert [p.material for p in sc] == [1.0] * 5 + [0.0]                  # REFLECTIVE.., MATTE
    assert sc[3].swizzle == rm.SWIZZLE_XZY                                # (pos - c).xzy, :119
    assert sc[5].paint == rm.PAINT_CHECKERS                               # checkers(pos), :121
    assert list(sc[0].center) == [15.0, 0.0, -10.0] and sc[0].param[0] == 3.0
    assert list(sc[2].param)[:4] == [3.0, 2.5, 2.5, 3.0]                  # box (3,2.5,2.5), r 3
    f = lambda x: float(np.float32(x))
    assert list(sc[4].param) == [f(-0.1), f(0.1), f(-0.1), 2.0, 4.0, 2.0, 1.0]
    assert list(sc[5].param)[:4] == [0.0, 1.0, 0.0, 5.5]
    assert [round(c, 4) for c in sc[1].color] == [0.0, 0.851, 1.0]


def test_default_scene_capacity(rm):
    n = C.c_int32(0)
    assert rm.lib().rm_default_scene(None, 0, C.byref(n)) == 0 and n.value == 6
    small = (rm.rm_primitive * 5)()
    assert rm.lib().rm_default_scene(small, 5, C.byref(n)) == rm.RM_ERR_INVALID
    assert C.sizeof(rm.rm_primitive) == 72


@pytest.mark.parametrize("frame,bounces,aa,shadow", [
    (0, 3, True, 0), (40, 5, False, 0), (119, 1, True, 1), (-1, 2, True, 0), (77, 0, False, 0)])
def test_oracle_table_mode_equals_the_glsl_scene(rm, oracle, frame, bounces, aa, shadow):
    u = rm.sweep_uniforms(frame, 120, bounces, aa, shadow)
    a = oracle.render(u, 64, 40)
    b = oracle.render(u, 64, 40, scene=rm.default_scene())
    np.testing.assert_array_equal(a["rgba32f"], b["rgba32f"])  # NaN == NaN here
    assert a["counters"] == b["counters"] and a["full_counters"] == b["full_counters"]
    np.testing.assert_array_equal(a["sdf_counts"], b["sdf_counts"])


def test_far_entries_change_nothing(rm, oracle):
    # an entry that is never the minimum leaves every sdf() value and id unchanged
    far = rm.primitive(rm.PRIM_SPHERE, (0.0, 5000.0, 0.0), (1.0,), (1, 0, 0), id=9)
    sc = rm.default_scene()
    u = rm.sweep_uniforms(30, 120, 2, False, 0)
    a = oracle.render(u, 48, 32, scene=sc)
    b = oracle.render(u, 48, 32, scene=sc + [far])
    c = oracle.render(u, 48, 32, scene=[far] + sc)
    np.testing.assert_array_equal(a["rgba32f"], b["rgba32f"])
    np.testing.assert_array_equal(a["rgba32f"], c["rgba32f"])


def test_scene_changes_the_image(rm, oracle):
    u = rm.sweep_uniforms(30, 120, 1, False, 0)
    sc = rm.default_scene()
    moved = rm.default_scene()
    moved[0].center[1] = 2.0                    # lift the green sphere
    a = oracle.render(u, 48, 32, scene=sc)["rgba8"]
    b = oracle.render(u, 48, 32, scene=moved)["rgba8"]
    assert (a != b).any()


def test_oracle_rejects_bad_tables(rm, oracle):
    u = rm.sweep_uniforms(0)
    out = np.zeros((4, 4, 4), np.uint8)
    L = oracle.lib()
    assert L.rmo_render_scene(C.byref(u), None, 0, 4, 4, None, 4, None, out.ctypes.data, None,
                              None, None, 1) == -1
    tbl = (rm.rm_primitive * 33)()
    assert L.rmo_render_scene(C.byref(u), tbl, 33, 4, 4, None, 4, None, out.ctypes.data, None,
                              None, None, 1) == -1


_CO_CACHE = {}


def _code_object(rm, scene, arch=b"gfx950"):
    """rm_jit_code_object: every call compiles, so one call with room to spare (a
    second, larger one only if the object outgrows it), cached per table."""
    tbl = (rm.rm_primitive * len(scene))(*scene)
    key = (bytes(tbl), arch)
    if key in _CO_CACHE:
        return _CO_CACHE[key]
    size = C.c_size_t(0)
    cap = 4 << 20
    buf = C.create_string_buffer(cap)
    rc = rm.lib().rm_jit_code_object(tbl, len(scene), arch, buf, cap, C.byref(size))
    if rc == rm.RM_ERR_INVALID and size.value > cap:
        buf = C.create_string_buffer(size.value)
        rc = rm.lib().rm_jit_code_object(tbl, len(scene), arch, buf, size.value, C.byref(size))
    out = (rc, buf.raw[:size.value] if rc == 0 else b"")
    _CO_CACHE[key] = out
    return out


def _kernel_private_sizes(co):
    """private_segment_fixed_size (scratch bytes per lane; u32 at offset 4 of the
    64-byte kernel descriptor `<kernel>.kd`) of every kernel in an AMDGPU ELF."""
    import struct
    shoff, = struct.unpack_from("<Q", co, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", co, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", co, shoff + i * shentsize) for i in range(shnum)]
    out = {}
    for name_, type_, flags, addr, off, size, link, info, align, entsize in secs:
        if type_ != 2:  # SHT_SYMTAB
            continue
        stroff = secs[link][4]
        for k in range(size // 24):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from(
                "<IBBHQQ", co, off + 24 * k)
            end = co.index(b"\0", stroff + st_name)
            sym = co[stroff + st_name:end].decode()
            if sym.endswith(".kd") and st_shndx < shnum:
                sec = secs[st_shndx]
                kd = sec[4] + (st_value - sec[3])
                out[sym[:-3]] = struct.unpack_from("<I", co, kd + 4)[0]
    return out


def test_table_specialises_without_a_device(rm):
    """rm_scene_specialize's hiprtc compile (rm_jit.hip) runs here, without a GPU:
    the embedded rm_table.hip compiles for gfx950 with the table folded in, and
    the code object holds the four table kernels.  The register bound (ADVICE r01,
    round 4): 8 waves per SIMD when the production kernels spill at most 32 B of
    scratch per lane there, else the most waves at which they need none; the
    kernel descriptors carry the private segment.  Round 6: the
    production kernels are the batch kernels, which also render single frames
    (a batch of one), and the reference scene's need no scratch at 8 waves."""
    rc, co = _code_object(rm, rm.default_scene())
    assert rc == 0 and co[:4] == b"\x7fELF"
    for name in (b"k_table_pixelILb1E", b"k_table_sampleILb1E", b"k_table_pixel_frames",
                 b"k_table_sample_frames"):
        assert name in co
    priv = _kernel_private_sizes(co)
    # the single-frame production kernels are not compiled (they spilled 12 B)
    assert not any("ILb0E" in k for k in priv), priv
    prod = {k: v for k, v in priv.items() if "_frames" in k}
    # (round 6: 0 B; round 5: 12 B in the single-frame kernel; round 4: 32 B)
    assert len(prod) == 2 and all(v == 0 for v in prod.values()), priv
    moved = rm.default_scene()
    moved[0].center[0] = 14.0
    rc2, co2 = _code_object(rm, moved)
    assert rc2 == 0 and co2 != co  # the table is compiled into the code
    bad = rm.default_scene()
    bad[0].type = 9
    assert _code_object(rm, bad)[0] == rm.RM_ERR_INVALID


def test_table_compiles_once(rm, tmp_path):
    """rm_scene_specialize compiles the reference scene's table once.
    The 8-wave build's kernel descriptors show at most 32 B of scratch per lane for
    the production kernels (64 VGPRs, 8 waves per SIMD), so no other bound is
    compiled; the hiprtc invocations are counted from RM_JIT_LOG's one line per
    compile."""
    import subprocess
    import sys
    prog = (
        "import ctypes as C, sys\n"
        f"sys.path.insert(0, {os.path.dirname(rm.__file__)!r}.rsplit('/', 1)[0])\n"
        "import rmarch as rm\n"
        "sc = rm.default_scene()\n"
        "tbl = (rm.rm_primitive * len(sc))(*sc)\n"
        "size = C.c_size_t(0)\n"
        "assert rm.lib().rm_jit_code_object(tbl, len(sc), b'gfx950', None, 0, C.byref(size)) == 0\n"
        "assert size.value > 0\n")
    out = subprocess.run([sys.executable, "-c", prog], env=dict(os.environ, RM_JIT_LOG="1"),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [x for x in out.stderr.splitlines() if x.startswith("rm_jit: hiprtc compile")]
    assert len(lines) == 1, out.stderr
    #  the log names the kernels that set the bound: the batch kernels
    bound = [x for x in out.stderr.splitlines() if x.startswith("rm_jit:   8-wave bound")]
    assert len(bound) == 2 and all("_frames" in x and " 0 B scratch" in x for x in bound), out.stderr
    rc, co = _code_object(rm, rm.default_scene())
    assert rc == 0
    vg = _kernel_vgprs(co)
    prod = {k: v for k, v in vg.items() if "_frames" in k}
    assert len(prod) == 2 and all(v <= 64 for v in prod.values()), vg  # 8 waves per SIMD


def test_large_tables_are_not_compiled(rm):
    """A table of more than 12 entries is not specialised and costs no hiprtc
    compile (a 16-entry table took 786 s of compiles to end on the generic kernel,
    rm_jit.hip kJitMaxEntries): *size = 0 at once, no compile logged."""
    import subprocess
    import sys
    prog = (
        "import ctypes as C, sys\n"
        f"sys.path.insert(0, {os.path.dirname(rm.__file__)!r}.rsplit('/', 1)[0])\n"
        "import rmarch as rm\n"
        "sc = rm.default_scene()\n"
        "sc = sc[:-1] * 3 + sc[-1:]\n"
        "assert len(sc) == 16\n"
        "for n in (13, 16):\n"
        "    t = sc[:n - 1] + sc[-1:]\n"
        "    tbl = (rm.rm_primitive * n)(*t)\n"
        "    size = C.c_size_t(1)\n"
        "    assert rm.lib().rm_jit_code_object(tbl, n, b'gfx950', None, 0, C.byref(size)) == 0\n"
        "    assert size.value == 0\n")
    out = subprocess.run([sys.executable, "-c", prog], env=dict(os.environ, RM_JIT_LOG="1"),
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "hiprtc compile" not in out.stderr, out.stderr


def _kernel_vgprs(co):
    """VGPR allocation per lane of every kernel (compute_pgm_rsrc1 bits 5:0 of its
    descriptor at offset 48: allocation / 8 - 1 on gfx950)."""
    import struct
    shoff, = struct.unpack_from("<Q", co, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", co, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", co, shoff + i * shentsize) for i in range(shnum)]
    out = {}
    for name_, type_, flags, addr, off, size, link, info, align, entsize in secs:
        if type_ != 2:
            continue
        stroff = secs[link][4]
        for k in range(size // 24):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from(
                "<IBBHQQ", co, off + 24 * k)
            end = co.index(b"\0", stroff + st_name)
            sym = co[stroff + st_name:end].decode()
            if sym.endswith(".kd") and st_shndx < shnum:
                sec = secs[st_shndx]
                kd = sec[4] + (st_value - sec[3])
                out[sym[:-3]] = ((struct.unpack_from("<I", co, kd + 48)[0] & 0x3F) + 1) * 8
    return out
