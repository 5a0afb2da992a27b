"""Hypothesis fuzz of the host table compiler: rm_scene_compile runs
rm::compile_scene and rm::exit_bounds exactly as rm_set_scene does, without a device.
Arbitrary rm_primitive tables (NaN, inf, huge and negative parameters, bad enums,
every size) must be refused or compiled into a well-formed table; for finite tables
of moderate size the culling balls and the exit ball must bound every entry's distance
(the soundness the table kernels' provable exits and lazy culling rest on,
rm_host.cpp exit_bounds).  tests/test_sanitizers.py runs this file under ASan + UBSan.
Reference: computeShader.glsl:83-123 (the primitives and opU)."""
import numpy as np
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

TABLE_WORDS, TW_TYPE, TW_BALL = 24, 0, 20
EX_VALID, EX_CX, EX_R, EX_NPLANES = 0, 1, 4, 7
EX_LIP, EX_NSLOTS, EX_EVAL_MASK, EX_PLANE_MASK, EX_SLOTS, EX_BOX, EXIT_WORDS = 24, 25, 26, 27, 28, 36, 42
PLANE = 5

f32_any = st.floats(width=32, allow_nan=True, allow_infinity=True)
f32_mid = st.floats(-60.0, 60.0, width=32)


def _prim(rm, draw_f, t, swz, paint, mat=1.0):
    return rm.primitive(t, tuple(draw_f() for _ in range(3)), tuple(draw_f() for _ in range(7)),
                        tuple(draw_f() for _ in range(3)), id=int(t), material=mat, swizzle=swz,
                        paint=paint)


@st.composite
def any_table(draw, rm):
    n = draw(st.integers(0, 34))
    prims = []
    for _ in range(n):
        t = draw(st.integers(-2, 7))
        swz = draw(st.integers(-1, 2))
        paint = draw(st.integers(-1, 2))
        prims.append(_prim(rm, lambda: draw(f32_any), t, swz, paint, mat=draw(f32_any)))
    return prims


@st.composite
def finite_table(draw, rm):
    n = draw(st.integers(1, 12))
    prims = []
    for _ in range(n):
        t = draw(st.integers(0, 5))
        prims.append(_prim(rm, lambda: draw(f32_mid), t, draw(st.integers(0, 1)), draw(st.integers(0, 1))))
    return prims


def _words(rm, prims):
    try:
        return rm.scene_words(prims)
    except rm.RMError as e:
        assert e.code == rm.RM_ERR_INVALID
        return None


def _f(w):
    return w.view(np.float32)


def _well_formed(prims, w):
    n = len(prims)
    assert w.shape == (n * TABLE_WORDS + EXIT_WORDS,)
    hdr = _f(w[n * TABLE_WORDS:])
    assert hdr[EX_VALID] in (0.0, 1.0)
    ns = int(hdr[EX_NSLOTS])
    assert 0 <= ns <= 8 and hdr[EX_NSLOTS] == ns
    slots = [int(v) for v in hdr[EX_SLOTS:EX_SLOTS + ns]]
    assert slots == sorted(set(slots)) and all(0 <= k < n for k in slots)
    assert all(prims[k].type != PLANE for k in slots)
    planes = {k for k in range(n) if prims[k].type == PLANE}
    assert int(w[n * TABLE_WORDS + EX_PLANE_MASK]) == sum(1 << k for k in planes)
    full = (1 << n) - 1 if n < 32 else 0xFFFFFFFF
    assert int(w[n * TABLE_WORDS + EX_EVAL_MASK]) == full & ~sum(1 << k for k in slots)
    for k in range(n):
        e = w[k * TABLE_WORDS:(k + 1) * TABLE_WORDS]
        assert int(e[TW_TYPE]) == prims[k].type
        ball = _f(e[TW_BALL:TW_BALL + 4])
        if hdr[EX_VALID] == 0.0 or prims[k].type == PLANE:
            assert ball[3] == np.inf, "no bound: never culled"
        else:
            assert np.isfinite(ball).all()
    if hdr[EX_VALID] == 1.0:
        assert 0 <= int(hdr[EX_NPLANES]) <= 4 and int(hdr[EX_NPLANES]) == len(planes)
        assert hdr[EX_LIP] >= 1.0


@settings(max_examples=400, deadline=None, suppress_health_check=list(HealthCheck))
@given(data=st.data())
def test_any_table_is_refused_or_well_formed(rm, data):
    prims = data.draw(any_table(rm))
    bad = (not 1 <= len(prims) <= 32 or any(
        p.type not in range(6) or p.swizzle not in (0, 1) or p.paint not in (0, 1) for p in prims))
    w = _words(rm, prims)
    assert (w is None) == bad
    if w is not None:
        _well_formed(prims, w)


def _sdf64(p, prim, blend):
    """One entry's distance in float64 (glsl:83-103, 115-121), q = swizzle(p - c)."""
    q = p - np.array(prim.center[:], np.float64)
    if prim.swizzle == 1:
        q = q[:, [0, 2, 1]]
    a = np.array(prim.param[:], np.float64)
    L = lambda v: np.sqrt((v * v).sum(-1))  # noqa: E731
    if prim.type == 0:
        return [L(q) - a[0]]
    if prim.type in (1, 2):
        d = np.abs(q) - a[:3]
        box = np.minimum(d.max(-1), 0.0) + L(np.maximum(d, 0.0))
        return [box] if prim.type == 1 else [box, L(q) - a[3]]  # a blend lies between the two
    if prim.type == 3:
        l2 = np.stack([L(q[:, [0, 2]]) - a[0], q[:, 1]], -1)
        return [L(l2) - a[1]]
    pa, ba = q - a[:3], a[3:6] - a[:3]
    h = np.clip((pa * ba).sum(-1) / (ba * ba).sum(), 0.0, 1.0)
    return [L(pa - ba * h[:, None]) - a[6]]


@settings(max_examples=250, deadline=None, suppress_health_check=list(HealthCheck))
@given(data=st.data())
def test_culling_balls_bound_every_entry(rm, data):
    """A valid table's per-entry ball (TW_BALL) and the table's exit ball (EX_C, EX_R)
    are lower bounds of the entries' distances: dist_k(p) >= |p - c_k| - r_k and the
    ball of every bounded entry lies inside the exit ball; so is the exit box (EX_BOX,
    the slab exits): dist_k(p) >= p_a - hi_a and lo_a - p_a on every axis."""
    prims = data.draw(finite_table(rm))
    w = _words(rm, prims)
    assert w is not None
    _well_formed(prims, w)
    n = len(prims)
    hdr = _f(w[n * TABLE_WORDS:]).astype(np.float64)
    if hdr[EX_VALID] != 1.0:
        return
    rng = np.random.default_rng(data.draw(st.integers(0, 2 ** 32 - 1)))
    p = rng.uniform(-150, 150, (64, 3))
    C, R = hdr[EX_CX:EX_CX + 3], hdr[EX_R]
    lo, hi = hdr[EX_BOX:EX_BOX + 3], hdr[EX_BOX + 3:EX_BOX + 6]
    slab = np.maximum(p - hi, lo - p).max(-1)
    for k, prim in enumerate(prims):
        if prim.type == PLANE:
            continue
        ball = _f(w[k * TABLE_WORDS + TW_BALL:k * TABLE_WORDS + TW_BALL + 4]).astype(np.float64)
        lb = np.sqrt(((p - ball[:3]) ** 2).sum(-1)) - ball[3]
        for d in _sdf64(p, prim, 0.5):
            ok = d >= lb - 1e-9 * (1.0 + np.abs(lb))
            assert ok.all(), (k, prim.type, (lb - d).max())
            ok = d >= slab - 1e-9 * (1.0 + np.abs(slab))
            assert ok.all(), (k, prim.type, (slab - d).max())
        assert np.sqrt(((ball[:3] - C) ** 2).sum()) + ball[3] <= R * (1 + 1e-6) + 1e-6, k
