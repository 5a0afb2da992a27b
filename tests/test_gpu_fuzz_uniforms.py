"""GPU parity on seeded random uniforms: cameras, view directions, lights, bounce
counts, AA and shadow modes the sweep and the stress list do not reach.

Each case: librm's counting build against the oracle (bit-exact geometry, RGBA8
within 1 LSB, RGBA32F within tolerance, NaN masks equal; test_gpu_parity's bar),
the production build (every proof-based early exit taken: the lazy culling
budgets, the ball / plane / slab / projection miss exits, the shadow exit,
rm_scene.hpp) equal to the counting build bit for bit, and finally every frame
once more through rm_dispatch_frames batches (k_sample_frames / k_pixel_frames,
the kernels bench.py times) equal to its single-frame image.

About a third of the cameras sit within 4 of a primitive's centre (some inside
it, where the reference itself yields NaN), a fifth of the lights are far away
(|light| ~ 1e3) and a fifth sit close to the objects.
"""
import os

import numpy as np
import pytest

from test_gpu_parity import _compare, _render_gpu

pytestmark = pytest.mark.gpu

SEED = 20261018
# RM_FUZZ_CASES widens the run (the first N cases do not depend on N)
NCASES = int(os.environ.get("RM_FUZZ_CASES", "256"))
W, H = 67, 41  # ragged: neither a multiple of the 8x8 tile

# primitive centres of the built-in scene (glsl:111-120; rm_scene.hpp offsets,
# CAP_M*): spheres, blend, torus, capsule midpoint
CENTRES = np.array([(15.0, 0.0, -10.0), (-25.0, 0.0, -10.0), (-5.0, 0.0, -10.0),
                    (-5.0, 0.0, 10.0), (-4.05, 0.05, -29.05)], np.float32)


def _cases():
    rng = np.random.default_rng(SEED)
    out = []
    for i in range(NCASES):
        if rng.random() < 0.35:
            pos = CENTRES[rng.integers(len(CENTRES))] + rng.uniform(-4.0, 4.0, 3)
        else:
            pos = rng.uniform((-40.0, -6.0, -40.0), (40.0, 15.0, 40.0))
        while True:
            look = np.array((-5.0, 0.0, -10.0)) + rng.uniform(-20.0, 20.0, 3)
            f = look - pos
            n = np.linalg.norm(f)
            if n > 1.0 and abs(f[1]) / n < 0.98:
                break
        r = rng.random()
        if r < 0.2:
            light = rng.uniform(-1.0, 1.0, 3) * 1.0e3
        elif r < 0.4:
            light = CENTRES[rng.integers(len(CENTRES))] + rng.uniform(-5.0, 5.0, 3)
        elif r < 0.8:
            light = rng.uniform((-40.0, -8.0, -40.0), (40.0, 30.0, 40.0))
        else:
            light = None  # the sweep's own light
        out.append(dict(pos=tuple(map(float, pos)), look=tuple(map(float, look)),
                        light=None if light is None else tuple(map(float, light)),
                        bounces=int(rng.integers(0, 6)), aa=bool(rng.random() < 0.5),
                        sm=int(rng.integers(0, 2)), itime=float(rng.uniform(0.0, 60.0)),
                        frame=int(rng.integers(0, 120))))
    return out


CASES = _cases()


def _uniforms(rm, c):
    u = rm.sweep_uniforms(c["frame"], 120, c["bounces"], c["aa"], c["sm"])
    u.camera = rm.Camera(W, H, pos=c["pos"], lookAt=c["look"]).to_uniform()
    if c["light"] is not None:
        for i in range(3):
            u.light.position[i] = c["light"][i]
    u.iTime = c["itime"]
    return u


_PROD = {}  # case index -> production image (RGBA32F, RGBA8), for the batch test


@pytest.mark.parametrize("i", range(NCASES))
def test_random_uniforms(rm, oracle, gpu, i):
    c = CASES[i]
    u = _uniforms(rm, c)
    ref = oracle.render(u, W, H)
    got = _render_gpu(rm, u, W, H, rm.RM_KERNEL_PIXEL)
    _compare(ref, got, f"case {i} {c}")
    prod = _render_gpu(rm, u, W, H, rm.RM_KERNEL_PIXEL, counters=False)
    np.testing.assert_array_equal(prod["rgba32f"], got["rgba32f"], err_msg=f"case {i}")
    np.testing.assert_array_equal(prod["rgba8"], got["rgba8"], err_msg=f"case {i}")
    _PROD[i] = (prod["rgba32f"], prod["rgba8"])


@pytest.mark.parametrize("aa", [False, True], ids=["noaa", "aa"])
def test_random_uniforms_batched(rm, gpu, aa):
    idx = [i for i, c in enumerate(CASES) if c["aa"] == aa]
    assert idx
    us = [_uniforms(rm, CASES[i]) for i in idx]
    with rm.Renderer(W, H, outputs=rm.RM_OUT_RGBA8 | rm.RM_OUT_RGBA32F,
                     kernel=rm.RM_KERNEL_PIXEL, counters=False) as r:
        single = {}
        for i, u in zip(idx, us):
            if i in _PROD:
                single[i] = _PROD[i]
            else:  # test_random_uniforms deselected: render the frame alone here
                r.dispatch(u)
                single[i] = (r.read_rgba32f(), r.read_rgba8())
        for b0 in range(0, len(idx), rm.RM_MAX_BATCH):
            bi, bu = idx[b0:b0 + rm.RM_MAX_BATCH], us[b0:b0 + rm.RM_MAX_BATCH]
            r.dispatch_frames(bu)
            r.synchronize()
            for k, i in enumerate(bi):
                np.testing.assert_array_equal(r.read_frame_rgba32f(k), single[i][0],
                                              err_msg=f"batch frame {k} (case {i})")
                np.testing.assert_array_equal(r.read_frame_rgba8(k), single[i][1],
                                              err_msg=f"batch frame {k} (case {i})")
