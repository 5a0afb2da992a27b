"""The provable-miss and shadow exits' object bounds (rm_scene.hpp lin_exit_b,
lin_exit_b3, lin_exit_b1p) against the reference
scene's five bounded primitives (rm_default_scene, float64 distances):

  * ball:       every object >= |p - C| - R_ALL                (C = (-5, 0, -10), R_ALL = 23.001)
  * slab:       every object >= p.y - SH_YTOP                  (SH_YTOP = 3.001)
  * projection: every object >= |rd| t + u - R_ALL along p(t) = ro + rd t,
                u = rd.(ro - C) / |rd|

The kernels' float roundings of the same bounds are covered by their margins
(stated in the code); this pins the geometry: the constants and the identity
|p(t) - C| >= |rd| t + u.  CPU only.
"""
import numpy as np
import pytest

from test_fuzz_tables import _sdf64

C = np.array([-5.0, 0.0, -10.0])
R_ALL = 23.001
SH_YTOP = 3.001


def _objects(rm, p):
    """min over the five bounded primitives (the blend as the lower of its box and
    sphere, which bounds every blend weight in [0, 1])."""
    prims = [q for q in rm.default_scene() if q.type != rm.PRIM_PLANE]
    assert len(prims) == 5
    return np.min([np.min(_sdf64(p, q, 0.5), axis=0) for q in prims], axis=0)


def test_ball_and_slab_bound_the_objects(rm):
    rng = np.random.default_rng(7)
    p = np.concatenate([rng.uniform(-60, 60, (200_000, 3)),
                        rng.uniform([-30, -4, -35], [20, 6, 15], (200_000, 3))])
    d = _objects(rm, p)
    assert (d >= np.linalg.norm(p - C, axis=1) - R_ALL - 1e-9).all()
    assert (d >= p[:, 1] - SH_YTOP).all()
    # the slab is tight: the objects reach y = 3 (a sphere top, the torus ring)
    assert abs(d[np.argmin(np.abs(p[:, 1] - 3.0) + np.abs(d))] - 0.0) < 0.5


def test_projection_bounds_the_objects_along_rays(rm):
    rng = np.random.default_rng(11)
    n = 4000
    ro = rng.uniform([-40, -5, -40], [30, 10, 20], (n, 3))
    rd = rng.normal(size=(n, 3)) * rng.uniform(0.5, 2.0, (n, 1))  # not unit: reflected rays
    rl = np.linalg.norm(rd, axis=1)
    u = ((ro - C) * rd).sum(1) / rl
    for t in (0.0, 0.5, 3.0, 10.0, 40.0, 150.0):
        p = ro + rd * t
        d = _objects(rm, p)
        assert (d >= rl * t + u - R_ALL - 1e-9).all(), t
        # and it is at least as tight as the triangle inequality's |rd| t - |ro - C|
        assert (rl * t + u >= rl * t - np.linalg.norm(ro - C, axis=1) - 1e-9).all()


# ---- the table exits' box (EX_BOX, rm_host.cpp exit_bounds) ------------------
# For every primitive type and swizzle, including the edge shapes the advisor named
# (negative sphere / torus radii, a blend whose sphere pokes out of its box, XZY-
# swizzled torus and capsule): every point on or inside the solid lies in the box
# rm_scene_compile returns, and at points outside the box the distance is at least the
# per-axis slab distance (what table_exit_T's slab exit relies on).
_BOX_CASES = [
    (0, (2.5,)), (0, (-1.5,)), (0, (0.0,)),
    (1, (3.0, 0.5, 1.25)), (1, (0.0, 2.0, 0.0)),
    (2, (3.0, 2.5, 2.5, 3.0)), (2, (1.0, 0.5, 0.25, 4.0)), (2, (3.0, 3.0, 3.0, 0.5)),
    (3, (2.5, 0.5)), (3, (1.0, 2.0)), (3, (-2.0, 0.5)), (3, (2.0, -0.25)),
    (4, (-1.0, -2.0, 0.5, 3.0, 4.0, -2.0, 1.0)), (4, (0.0, 0.0, 0.0, 0.0, 6.0, 0.0, 0.75)),
]


@pytest.mark.parametrize("swz", [0, 1])
@pytest.mark.parametrize("case", range(len(_BOX_CASES)))
def test_exit_box_holds_every_solid(rm, case, swz):
    from test_fuzz_tables import EX_BOX, EX_VALID, TABLE_WORDS, _f
    t, param = _BOX_CASES[case]
    center = (-4.0, 1.5, -9.0)
    prim = rm.primitive(t, center, param, (0.5, 0.5, 0.5), id=1, swizzle=swz)
    floor = rm.primitive(rm.PRIM_PLANE, (0.0, 0.0, 0.0), (0.0, 1.0, 0.0, 5.5), id=7, material=0.0)
    w = rm.scene_words([prim, floor])
    hdr = _f(w[2 * TABLE_WORDS:]).astype(np.float64)
    if hdr[EX_VALID] != 1.0:
        pytest.skip("the host gives this table no exit bounds (exits off): nothing to check")
    lo, hi = hdr[EX_BOX:EX_BOX + 3], hdr[EX_BOX + 3:EX_BOX + 6]
    assert (lo <= hi).all()
    rng = np.random.default_rng(100 + case + 50 * swz)
    ext = 1.5 * (np.abs(np.array(param)).sum() + 1.0)
    # three scales around the centre, so thin and small solids get inside points too
    p = np.array(center) + np.concatenate([rng.uniform(-e, e, (200_000, 3)) for e in (ext, ext / 4, ext / 16)])
    # a blend is inside for some weight (sin(iTime) moves it) where its box or its
    # sphere is: the box must hold both
    d = np.min(_sdf64(p, prim, 0.5), axis=0)
    inside = p[d <= 0.0]
    empty = ((t == 0 and param[0] <= 0.0) or (t == 1 and min(param[:3]) <= 0.0)
             or (t == 2 and min(param[:3]) <= 0.0 and param[3] <= 0.0)
             or (t == 3 and (param[1] <= 0.0 or -param[0] > param[1])))
    if empty:
        assert len(inside) == 0, "an empty solid: its distance is positive everywhere sampled"
    else:
        assert len(inside) > 100, "the sampler found the solid"
    tol = 1e-9 * (1.0 + np.abs(p).max())
    assert (inside >= lo - tol).all() and (inside <= hi + tol).all(), (lo, hi, inside.min(0), inside.max(0))
    # outside the box: every blend weight's distance is at least the slab distance
    slab = np.maximum(p - hi, lo - p).max(-1)
    out = slab > 0
    dmin = np.min(_sdf64(p[out], prim, 0.5), axis=0)
    assert (dmin >= slab[out] - 1e-9 * (1.0 + slab[out])).all()
