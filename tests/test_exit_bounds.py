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
