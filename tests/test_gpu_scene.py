"""Runtime scene table on the GPU, through the C-ABI.

  * the reference scene as a table (rm_default_scene) renders the same image as the
    built-in scene's specialised kernel, bit for bit in RGBA32F, with identical
    per-pixel sdf() counts and frame counters;
  * random tables (every primitive type, swizzle, paint, MATTE entries, id-7 floor
    entries) match the oracle's table mode with the bar of test_gpu_parity.py:
    geometry (sdf counts, counters) exact, RGBA8 within 1 LSB;
  * graph replay, row shards, switching back to the built-in scene and argument
    validation behave as for the built-in scene.
"""
import ctypes as C

import numpy as np
import pytest

from test_gpu_parity import _compare

pytestmark = pytest.mark.gpu

OUT = 3  # RGBA8 | RGBA32F


def _render(rm, u, W, H, scene=None, counters=True, **kw):
    with rm.Renderer(W, H, outputs=OUT, counters=counters, **kw) as r:
        if scene is not None:
            r.set_scene(scene)
        r.dispatch(u)
        out = {"rgba8": r.read_rgba8(), "rgba32f": r.read_rgba32f()}
        if counters:
            out["counters"] = r.counters()
            out["sdf_counts"] = r.sdf_counts()
    return out


CASES = [(-1, 0, True, 0), (0, 0, False, 1), (60, 1, False, 0), (0, 3, True, 0),
         (119, 3, True, 0), (60, 5, True, 0), (90, 4, False, 0)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"f{c[0]}_b{c[1]}_aa{int(c[2])}_s{c[3]}")
def test_default_table_equals_builtin_kernel(rm, gpu, case):
    f, b, aa, sm = case
    u = rm.sweep_uniforms(f, 120, b, aa, sm)
    W, H = 160, 96
    for counters in (True, False):
        ref = _render(rm, u, W, H, counters=counters)
        got = _render(rm, u, W, H, scene=rm.default_scene(), counters=counters)
        np.testing.assert_array_equal(got["rgba32f"], ref["rgba32f"])
        np.testing.assert_array_equal(got["rgba8"], ref["rgba8"])
        if counters:
            assert got["counters"] == ref["counters"]
            np.testing.assert_array_equal(got["sdf_counts"], ref["sdf_counts"])


def test_default_table_equals_builtin_kernel_full_hd(rm, gpu):
    u = rm.sweep_uniforms(45, 120, 3, True, 0)
    ref = _render(rm, u, 1920, 1080, counters=False)
    got = _render(rm, u, 1920, 1080, scene=rm.default_scene(), counters=False)
    np.testing.assert_array_equal(got["rgba32f"], ref["rgba32f"])


def random_scene(rm, seed, nplanes=None):
    """Random table; nplanes fixes the number of plane entries (None: random types)."""
    g = np.random.default_rng(seed)
    n = int(g.integers(3, 13))
    types = [int(g.integers(0, 6)) for _ in range(n)]
    if nplanes is not None:
        types = [int(g.integers(0, 5)) for _ in range(n)] + [rm.PRIM_PLANE] * nplanes
        g.shuffle(types)
    prims = []
    for t in types:
        c = (float(g.uniform(-18, 18)), float(g.uniform(-3, 3)), float(g.uniform(-35, 0)))
        if t == rm.PRIM_SPHERE:
            par = (float(g.uniform(0.5, 4)),)
        elif t == rm.PRIM_BOX:
            par = tuple(float(x) for x in g.uniform(0.3, 3, 3))
        elif t == rm.PRIM_BLEND:
            par = tuple(float(x) for x in g.uniform(0.3, 3, 3)) + (float(g.uniform(0.5, 3)),)
        elif t == rm.PRIM_TORUS:
            par = (float(g.uniform(1, 3)), float(g.uniform(0.2, 0.8)))
        elif t == rm.PRIM_CAPSULE:
            par = tuple(float(x) for x in g.uniform(-2, 2, 6)) + (float(g.uniform(0.3, 1.5)),)
        else:
            nv = g.normal(size=3)
            nv[1] = abs(nv[1]) + 1.0
            if nplanes is not None and g.uniform() < 0.5:
                nv[1] = -nv[1]  # a ceiling: rays going up meet it, the miss exit must not fire
            nv /= np.linalg.norm(nv)
            c = (0.0, 0.0, 0.0)
            par = (float(nv[0]), float(nv[1]), float(nv[2]), float(g.uniform(4, 7)))
        prims.append(rm.primitive(
            t, c, par, tuple(float(x) for x in g.uniform(0, 1, 3)),
            id=int(g.choice([0, 1, 2, 5, 7, 7, 9])),
            material=float(g.choice([1.0, 1.0, 0.0])),
            swizzle=int(g.integers(0, 2)),
            paint=int(g.choice([0, 0, 1]))))
    return prims


@pytest.mark.parametrize("seed", range(8))
def test_random_tables_match_oracle(rm, oracle, gpu, seed):
    scene = random_scene(rm, seed)
    f, b, aa, sm = [(10, 2, True, 0), (60, 3, False, 0), (100, 5, True, 1), (30, 1, False, 0)][seed % 4]
    u = rm.sweep_uniforms(f, 120, b, aa, sm)
    W, H = 96, 64
    ref = oracle.render(u, W, H, scene=scene)
    got = _render(rm, u, W, H, scene=scene)
    _compare(ref, got, f"seed {seed}")
    prod = _render(rm, u, W, H, scene=scene, counters=False)
    np.testing.assert_array_equal(prod["rgba32f"], got["rgba32f"])


def test_switching_scenes(rm, gpu):
    u = rm.sweep_uniforms(20, 120, 2, False, 0)
    with rm.Renderer(64, 48, outputs=OUT) as r:
        assert r.get_scene() == []
        r.dispatch(u)
        a = r.read_rgba32f()
        moved = rm.default_scene()
        moved[2].center[0] = 0.0
        r.set_scene(moved)
        assert [p.center[0] for p in r.get_scene()] == [p.center[0] for p in moved]
        r.dispatch(u)
        b = r.read_rgba32f()
        r.set_scene(None)
        r.dispatch(u)
        c = r.read_rgba32f()
    assert (a != b).any()
    np.testing.assert_array_equal(a, c)


def test_table_validation(rm, gpu):
    with rm.Renderer(16, 16) as r:
        bad = rm.default_scene()
        bad[1].type = 9
        with pytest.raises(rm.RMError):
            r.set_scene(bad)
        bad = rm.default_scene()
        bad[0].swizzle = 3
        with pytest.raises(rm.RMError):
            r.set_scene(bad)
        with pytest.raises(rm.RMError):
            r.set_scene(rm.default_scene() * 6)  # 36 > RM_MAX_PRIMITIVES
        assert rm.lib().rm_set_scene(r.handle, None, 3) == rm.RM_ERR_INVALID
        assert r.get_scene() == []  # failed calls leave the scene unchanged


def test_table_graph_replay(rm, gpu):
    sc = rm.default_scene()
    sc[0].center[1] = 1.5
    frames = [rm.sweep_uniforms(f, 120, 3, aa, 0) for f, aa in ((0, True), (50, True), (90, False))]
    want = []
    with rm.Renderer(80, 48, outputs=OUT) as r:
        r.set_scene(sc)
        for u in frames:
            r.dispatch(u)
            want.append(r.read_rgba32f())
    with rm.Renderer(80, 48, outputs=OUT) as r:
        r.set_scene(sc)
        r.graph_enable(True)
        for u, w in zip(frames, want):
            r.graph_dispatch(u)
            np.testing.assert_array_equal(r.read_rgba32f(), w)
        r.set_scene(None)  # re-captures the built-in kernel
        r.graph_dispatch(frames[0])
        ref = _render(rm, frames[0], 80, 48, counters=False)
        np.testing.assert_array_equal(r.read_rgba32f(), ref["rgba32f"])


@pytest.mark.parametrize("R0", [4, 3])
def test_table_shards_assemble(rm, gpu, R0):
    W, H, N, R = 64, 50, 3, 4
    sc = random_scene(rm, 3)
    u = rm.sweep_uniforms(40, 120, 2, True, 0)
    full = _render(rm, u, W, H, scene=sc, counters=False)["rgba8"]
    cap = C.c_int32(0)
    rm.lib().rm_shard_rows(H, R, R0, N, 0, None, C.byref(cap))
    parts = []
    for s in range(N):
        with rm.Renderer(W, H, row_block=R, shard=s, nshards=N, rank0_rows=R0) as r:
            r.set_scene(sc)
            r.dispatch(u)
            parts.append(r.read_rgba8())
    got = np.zeros_like(full)
    for s in range(N):
        for lr in range(cap.value):
            g = rm.lib().rm_shard_to_global(H, R, R0, N, s, lr)
            if g >= 0:
                got[g] = parts[s][lr]
    np.testing.assert_array_equal(got, full)


# The table kernels' provable early exits (rm_table.hip table_exit_T) on tables
# without a plane (sky rays leave through the ball bound alone), with several
# floor / ceiling planes, and with more planes than the exit header holds (exits
# off).  The counting build runs every step and poisons a proven miss that hits
# (NaN), so the counts, images and NaN masks check the proofs.
@pytest.mark.parametrize("seed,nplanes", [(100, 0), (101, 0), (102, 2), (103, 3), (104, 1), (105, 5)])
def test_table_exits_match_oracle(rm, oracle, gpu, seed, nplanes):
    scene = random_scene(rm, seed, nplanes=nplanes)
    f, b, aa, sm = [(20, 3, True, 0), (70, 2, False, 0), (110, 4, True, 1)][seed % 3]
    u = rm.sweep_uniforms(f, 120, b, aa, sm)
    W, H = 96, 64
    ref = oracle.render(u, W, H, scene=scene)
    got = _render(rm, u, W, H, scene=scene)
    _compare(ref, got, f"seed {seed}")
    prod = _render(rm, u, W, H, scene=scene, counters=False)
    np.testing.assert_array_equal(prod["rgba32f"], got["rgba32f"])


# Specialised table kernels (rm_scene_specialize: hiprtc compiles rm_table.hip
# for the table itself, rm_jit.hip).  Same source and flags, so the images,
# counters and per-pixel sdf counts must equal the generic table kernel's (and,
# for the reference scene, the built-in kernel's) bit for bit.
def _render_spec(rm, u, W, H, scene, counters=True, **kw):
    with rm.Renderer(W, H, outputs=OUT, counters=counters, **kw) as r:
        r.specialize_scene(True)
        r.set_scene(scene)
        r.dispatch(u)
        out = {"rgba8": r.read_rgba8(), "rgba32f": r.read_rgba32f()}
        if counters:
            out["counters"] = r.counters()
            out["sdf_counts"] = r.sdf_counts()
    return out


def _same(a, b):
    np.testing.assert_array_equal(a["rgba32f"], b["rgba32f"])
    np.testing.assert_array_equal(a["rgba8"], b["rgba8"])
    if "counters" in a:
        assert a["counters"] == b["counters"]
        np.testing.assert_array_equal(a["sdf_counts"], b["sdf_counts"])


@pytest.mark.parametrize("case", CASES[:5], ids=lambda c: f"f{c[0]}_b{c[1]}_aa{int(c[2])}_s{c[3]}")
def test_specialised_default_table_equals_builtin(rm, gpu, case):
    f, b, aa, sm = case
    u = rm.sweep_uniforms(f, 120, b, aa, sm)
    for counters in (True, False):
        _same(_render_spec(rm, u, 160, 96, rm.default_scene(), counters=counters),
              _render(rm, u, 160, 96, counters=counters))


@pytest.mark.parametrize("seed,nplanes", [(4, None), (5, None), (6, None), (102, 2), (105, 5)])
def test_specialised_tables_equal_generic(rm, gpu, seed, nplanes):
    scene = random_scene(rm, seed, nplanes=nplanes)
    f, b, aa, sm = [(10, 2, True, 0), (60, 3, False, 0), (100, 5, True, 1)][seed % 3]
    u = rm.sweep_uniforms(f, 120, b, aa, sm)
    for counters in (True, False):
        _same(_render_spec(rm, u, 96, 64, scene, counters=counters),
              _render(rm, u, 96, 64, scene=scene, counters=counters))


def floor_last_scene(rm, seed):
    """A reference-shaped table (the specialised kernel's built-in-style march,
    rm_table.hip smarch): random bounded entries, then one axis-aligned floor
    plane q.y n_y + w as the last entry, n_y of either sign and not unit."""
    g = np.random.default_rng(1000 + seed)
    # 3..7 bounded entries (every one in a lazy slot): the 5- and 8-slot instances
    prims = random_scene(rm, seed, nplanes=0)[:3 + seed % 5]
    ny = float(g.choice([1.0, 0.5, 2.0, -1.0]))  # -1: a ceiling above the scene
    w = float(g.uniform(4, 7)) * abs(ny)
    prims.append(rm.primitive(rm.PRIM_PLANE, (0.0, 0.0, 0.0), (0.0, ny, 0.0, w), (0.5, 0.5, 0.5),
                              id=7, material=0.0, paint=1))
    return prims


@pytest.mark.parametrize("seed", range(6))
def test_specialised_floor_tables_equal_generic(rm, gpu, seed):
    """Reference-shaped tables take the specialised kernels' lazy block (plane
    budget, slack line, bounded sqrt form): the same image, counters and sdf
    counts as the generic kernel."""
    scene = floor_last_scene(rm, seed)
    f, b, aa, sm = [(10, 2, True, 0), (60, 3, False, 0), (100, 5, True, 1)][seed % 3]
    u = rm.sweep_uniforms(f, 120, b, aa, sm)
    for counters in (True, False):
        _same(_render_spec(rm, u, 96, 64, scene, counters=counters),
              _render(rm, u, 96, 64, scene=scene, counters=counters))


@pytest.mark.parametrize("seed", range(6))
def test_floor_tables_match_oracle(rm, oracle, gpu, seed):
    """Reference-shaped tables through the generic kernel: the counting kernel
    (TLazy) against the oracle's table mode, and the production kernel's
    reference-shaped instance (smarch, 5 or 8 slots) against the counting image
    bit for bit."""
    scene = floor_last_scene(rm, seed)
    f, b, aa, sm = [(10, 2, True, 0), (60, 3, False, 0), (100, 5, True, 1), (30, 1, False, 0)][seed % 4]
    u = rm.sweep_uniforms(f, 120, b, aa, sm)
    W, H = 96, 64
    ref = oracle.render(u, W, H, scene=scene)
    got = _render(rm, u, W, H, scene=scene)
    _compare(ref, got, f"floor seed {seed}")
    prod = _render(rm, u, W, H, scene=scene, counters=False)
    np.testing.assert_array_equal(prod["rgba32f"], got["rgba32f"])


def test_specialised_far_camera_uses_generic(rm, gpu):
    """A camera farther than 1e15 from the origin is outside the specialised
    kernels' bounded-point assumption (rm_api.hip frame_jit): the frame renders
    with the generic kernel, and graph replay re-captures both ways."""
    near = rm.sweep_uniforms(60, 120, 3, True, 0)
    far = rm.sweep_uniforms(60, 120, 3, True, 0)
    far.camera.pos[0] = 3e15
    want = {k: _render(rm, u, 64, 48, scene=rm.default_scene(), counters=False)["rgba32f"]
            for k, u in (("near", near), ("far", far))}
    with rm.Renderer(64, 48, outputs=OUT) as r:
        r.specialize_scene(True)
        r.set_scene(rm.default_scene())
        for k, u in (("near", near), ("far", far), ("near", near)):
            r.dispatch(u)
            np.testing.assert_array_equal(r.read_rgba32f(), want[k])
        r.graph_enable(True)
        for k, u in (("far", far), ("near", near), ("far", far)):
            r.graph_dispatch(u)
            np.testing.assert_array_equal(r.read_rgba32f(), want[k])


@pytest.mark.parametrize("lx", [1e15, 1e30, 3e38])
def test_specialised_far_light_equals_generic(rm, gpu, lx):
    """the light position is a free uniform and shadow rays are
    light - pos, unnormalised (glsl:184, 235), so with a light near FLT_MAX shadow
    points overflow.  The specialised kernels' shadow march takes the full-range
    sqrt (as the generic kernel), so far lights, inf and NaN included, render the
    generic kernel's image bit for bit (camera near: the specialised kernels run)."""
    for scene in (rm.default_scene(), floor_last_scene(rm, 2)):
        for sm in (0, 1):
            u = rm.sweep_uniforms(60, 120, 3, True, sm)
            u.light.position[0] = lx
            u.light.position[1] = lx / 3
            _same(_render_spec(rm, u, 64, 48, scene, counters=False),
                  _render(rm, u, 64, 48, scene=scene, counters=False))


def test_specialise_toggle_and_graph(rm, gpu):
    """Toggling specialisation and switching tables re-captures the graph."""
    a, b = rm.default_scene(), random_scene(rm, 7)
    frames = [rm.sweep_uniforms(f, 120, 3, True, 0) for f in (0, 60)]
    want = {}
    for name, sc in (("a", a), ("b", b)):
        for i, u in enumerate(frames):
            want[name, i] = _render(rm, u, 80, 48, scene=sc, counters=False)["rgba32f"]
    with rm.Renderer(80, 48, outputs=OUT) as r:
        r.set_scene(a)
        r.specialize_scene(True)  # compiles for the current table
        r.graph_enable(True)
        for i, u in enumerate(frames):
            r.graph_dispatch(u)
            np.testing.assert_array_equal(r.read_rgba32f(), want["a", i])
        r.set_scene(b)  # compiles b; the graph holds a's kernel and must re-capture
        for i, u in enumerate(frames):
            r.graph_dispatch(u)
            np.testing.assert_array_equal(r.read_rgba32f(), want["b", i])
        r.specialize_scene(False)  # back to the generic kernel
        r.graph_dispatch(frames[1])
        np.testing.assert_array_equal(r.read_rgba32f(), want["b", 1])
        r.set_scene(a)
        r.specialize_scene(True)  # the cached module: no second compile
        r.dispatch(frames[0])
        np.testing.assert_array_equal(r.read_rgba32f(), want["a", 0])


def _big_table(rm, n=30):
    """The reference scene's 5 objects repeated along x (40 units apart), one plane."""
    import ctypes as C
    out = []
    for k in range(8):
        for p in rm.default_scene():
            if p.type == rm.PRIM_PLANE and k:
                continue
            q = rm.rm_primitive()
            C.memmove(C.byref(q), C.byref(p), C.sizeof(p))
            if q.type != rm.PRIM_PLANE:
                q.center[0] += 40.0 * k
            out.append(q)
    return out[:n]


def test_specialisation_register_bound(rm, gpu):
    """rm_jit.hip compiles a table for the most waves per SIMD (8, 7, 6) at which
    its production kernels need no scratch (one fixed 8-wave bound
    spilled for the reference scene and spilled hundreds of VGPRs for large
    tables).  The reference scene specialises; a 30-entry table is not compiled
    (more than 12 entries, rm_jit.hip kJitMaxEntries) and renders with the generic
    kernel, with the same image."""
    u = rm.sweep_uniforms(60, 120, 3, True, 0)
    with rm.Renderer(96, 64, outputs=OUT) as r:
        assert r.scene_kernel_waves() == 0  # built-in scene
        r.specialize_scene(True)
        r.set_scene(rm.default_scene())
        assert r.scene_kernel_waves() in (6, 7, 8)
        big = _big_table(rm)
        assert len(big) == 30
        r.set_scene(big)
        assert r.scene_kernel_waves() == 0
        r.dispatch(u)
        got = r.read_rgba32f()
    want = _render(rm, u, 96, 64, scene=big, counters=False)["rgba32f"]
    np.testing.assert_array_equal(got, want)


# Tables that are not reference-shaped: several planes, the floor
# not last, a tilted floor, more bounded entries than the lazy slots.  Their
# production kernels march with the block shape of any plane-bounded table
# (rm_table.hip gmarch); the counting kernels keep TLazy.
@pytest.mark.parametrize("shape", ["planes2", "plane_mid", "tilted", "many"])
def test_table_shapes_match_oracle(rm, oracle, gpu, shape):
    """The counting kernel against the oracle's table mode (exact counts, <= 1 LSB),
    the production kernel (gmarch) bit-equal to the counting image, and the
    specialised kernels (gmarch unrolled over the table) bit-equal to the generic."""
    import os
    from tools.probe_table_shapes import shape_table
    sc = shape_table(shape)
    W, H = 96, 64
    if shape == "many":
        # ten entries need three hiprtc compiles to find their bound (~2.5 min on
        # the box's CPU); the 6-wave bound the ladder ends at, in one compile
        os.environ["RM_JIT_FORCE_WAVES"] = "6"
    for f, b, aa, sm in [(30, 3, True, 0), (90, 2, False, 1), (5, 5, True, 0)]:
        u = rm.sweep_uniforms(f, 120, b, aa, sm)
        ref = oracle.render(u, W, H, scene=sc)
        got = _render(rm, u, W, H, scene=sc)
        _compare(ref, got, f"{shape} f{f}")
        prod = _render(rm, u, W, H, scene=sc, counters=False)
        np.testing.assert_array_equal(prod["rgba32f"], got["rgba32f"])
        try:
            _same(_render_spec(rm, u, W, H, sc, counters=False), prod)
        finally:
            os.environ.pop("RM_JIT_FORCE_WAVES", None)
